#!/bin/bash
# Round-2 GPU session: full -m gpu suite, smoke, default bench, every secondary workload's bench line
# (PowerSGD / sign over 200 steps: their steps are tens of microseconds), rocprof kernel stats of
# the default workload.  Each GPU step has its own time limit; a crash / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for step in ${STEPS:-pytest smoke bench secondary prof}; do
  case $step in
    pytest) run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python3 bench.py ;;
    secondary)
      : > gpurun_out/secondary.jsonl
      for wl in ${WL:-sign sign256 qsgd terngrad powersgd topk_sharded topk_e2e ddp_params ddp_segmented ddp_bucket}; do
        st=20; case $wl in sign|powersgd|ddp_segmented) st=200;; esac
        run "bench_$wl" 300 python3 bench.py --workload $wl --steps $st --no-cpu-baseline
        grep '^{' "gpurun_out/bench_$wl.log" | tail -1 >> gpurun_out/secondary.jsonl
      done ;;
    prof) run prof_topk 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02_topk -o run \
            -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
  esac
done
