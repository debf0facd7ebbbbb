set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_sharded.py tests/test_gpu_dgc.py -x -q > gpurun_out/pysh.log 2>&1; rc=$?; tail -5 gpurun_out/pysh.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/exp_psgd.py > gpurun_out/expp.log 2>&1 || exit $?
BENCH_WL="topk_sharded" bash tools/gpu_session.sh benchall && PROF_WL="topk_sharded" SESSION_TAG=r01q bash tools/gpu_session.sh profwl
