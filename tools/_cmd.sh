set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_sparse.py -x -q -k aggregate > gpurun_out/pyt.log 2>&1; rc=$?; tail -3 gpurun_out/pyt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_w8b -o w8 -- python3 $GRAFT_REPO_ROOT/tools/exp_w8.py > gpurun_out/w8p.log 2>&1 || exit $?
