#!/bin/bash
# Round-2 profile session on the GPU box: kernel-trace stats of every bench workload, then
# FETCH_SIZE / WRITE_SIZE passes (one counter per run) for the secondary workloads.  Each GPU step
# has its own time limit; the first crash / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02}
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "gpurun_out/$name.log"; exit $rc; fi; }
for wl in ${PROF_WL:-topk qsgd terngrad powersgd sign sign256}; do
  run "stats_$wl" 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_${TAG}_$wl" -o run \
      -- python3 bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline
done
for wl in ${PMC_WL:-qsgd terngrad powersgd sign256}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$c" 120 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_${TAG}_${wl}_$c" -o pmc \
        -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline
  done
done
args=""
for wl in ${PMC_WL:-qsgd terngrad powersgd sign256}; do args="$args $wl=gpurun_out/pmc_${TAG}_${wl}_FETCH_SIZE,gpurun_out/pmc_${TAG}_${wl}_WRITE_SIZE"; done
python3 tools/pmc_all.py gpurun_out/pmc_${TAG}_secondary.json $args
