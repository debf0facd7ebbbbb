set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pyall.log 2>&1; rc=$?; tail -5 gpurun_out/pyall.log; [ $rc -le 1 ] || exit $rc
BENCH_WL="qsgd terngrad powersgd sign sign256" bash tools/gpu_session.sh benchall && bash tools/gpu_session.sh bench
