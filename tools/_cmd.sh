set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=grace_amd/lib
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_powersgd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { tail -40 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
timeout -k 10 400 python3 tools/exp_psgd.py $L/libgrace_hip.so $L/libgrace_hip_psa.so $L/libgrace_hip_psb.so $L/libgrace_hip_psc.so $L/libgrace_hip_psd.so $L/libgrace_hip.so > gpurun_out/psgd.log 2>&1 || { tail -20 gpurun_out/psgd.log; exit 1; }
cat gpurun_out/psgd.log
