set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_dgc.py -x -q > gpurun_out/pydgc.log 2>&1; rc=$?; tail -5 gpurun_out/pydgc.log; [ $rc -le 1 ] || exit $rc
SESSION_TAG=r01p bash tools/gpu_session.sh prof && PROF_WL="powersgd topk_sharded" SESSION_TAG=r01p bash tools/gpu_session.sh profwl
