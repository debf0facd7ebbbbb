set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python3 -m pytest tests -m gpu -x -q > gpurun_out/pyall.log 2>&1; rc=$?; tail -5 gpurun_out/pyall.log; [ $rc -le 1 ] || exit $rc
