set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_topk.py tests/test_gpu_dgc.py tests/test_gpu_world2.py tests/test_gpu_harness.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { tail -40 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
timeout -k 10 300 python3 tools/exp_fallback.py > gpurun_out/fb.log 2>&1 || { tail -20 gpurun_out/fb.log; exit 1; }
cat gpurun_out/fb.log
