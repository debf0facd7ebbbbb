set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_powersgd.py tests/test_gpu_quant.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { tail -30 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_p -o q -- python3 $GRAFT_REPO_ROOT/bench.py --workload powersgd --steps 20 > gpurun_out/p.log 2>&1 || exit $?
tail -1 gpurun_out/p.log | cut -c1-200
timeout -k 10 120 python3 bench.py --workload sign --steps 200 > gpurun_out/s.log 2>&1 || exit $?
tail -1 gpurun_out/s.log | cut -c1-200
