set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
BENCH_WL="powersgd" bash tools/gpu_session.sh pytest bench benchall
timeout -k 10 300 python3 tools/exp_fallback.py > gpurun_out/fb.log 2>&1 || { tail -20 gpurun_out/fb.log; exit 1; }
cat gpurun_out/fb.log
