set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_topk.py tests/test_gpu_sharded.py -x -q > gpurun_out/pyt.log 2>&1; rc=$?; tail -3 gpurun_out/pyt.log; [ $rc -le 1 ] || exit $rc
L=grace_amd/lib
timeout -k 10 600 python3 tools/ab_topk.py $L/libgrace_hip.so $L/libgrace_hip_s1.so $L/libgrace_hip_v8.so $L/libgrace_hip_v32.so $L/libgrace_hip_g2.so $L/libgrace_hip_g8.so $L/libgrace_hip_b512.so > gpurun_out/ab.log 2>&1 || exit $?
SESSION_TAG=r01r bash tools/gpu_session.sh prof
