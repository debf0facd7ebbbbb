set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=grace_amd/lib
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_topk.py tests/test_gpu_sharded.py tests/test_gpu_dgc.py tests/test_gpu_world2.py tests/test_gpu_harness.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { tail -30 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
timeout -k 10 300 python3 tools/ab_topk.py $L/libgrace_hip_head.so $L/libgrace_hip.so $L/libgrace_hip_head.so $L/libgrace_hip.so > gpurun_out/ab.log 2>&1 || exit $?
cat gpurun_out/ab.log
