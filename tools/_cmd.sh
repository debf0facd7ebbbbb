set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_sharded.py tests/test_gpu_topk.py tests/test_gpu_world2.py -x -q > gpurun_out/pysh.log 2>&1; rc=$?; tail -5 gpurun_out/pysh.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_session.sh bench
