set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_w8 -o w8 -- python3 $GRAFT_REPO_ROOT/tools/exp_w8.py > gpurun_out/w8p.log 2>&1 || exit $?
