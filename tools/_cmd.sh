set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_harness.py -x -q > gpurun_out/pyh.log 2>&1; rc=$?; tail -3 gpurun_out/pyh.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_session.sh smoke bench benchall
