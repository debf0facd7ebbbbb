#!/bin/bash
# r05 PMC session (copy of pmc_r03.sh with r05 names): FETCH_SIZE / WRITE_SIZE passes (one counter per run, each under its own kill
# timeout, in-bench probes off) for the headline top-k step and the secondary workloads, then the
# per-step summaries bench.py reads (profiles/pmc_topk_main.json, profiles/r05_pmc_secondary.json
# once copied from gpurun_out/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GRACE_BENCH_NO_PROBE=1
run() { local name=$1; shift; echo "== $name"; timeout -s KILL 90 "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "gpurun_out/$name.log"; exit $rc; fi; }
if [ -z "${SKIP_HEAD:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc_head_$c" rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_r05_topk_$c" -o pmc \
        -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-overlap
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_r05_topk_FETCH_SIZE gpurun_out/pmc_r05_topk_WRITE_SIZE \
      "topk_main<true" 67108864 1 gpurun_out/pmc_topk_main.json
fi
args=""
for wl in ${PMC_WL:-qsgd terngrad powersgd sign256 qsgd_step terngrad_step topk_sharded ddp_segmented randomk threshold dgc topk_nomem}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$c" rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_r05_${wl}_$c" -o pmc \
        -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline
  done
  args="$args $wl=gpurun_out/pmc_r05_${wl}_FETCH_SIZE,gpurun_out/pmc_r05_${wl}_WRITE_SIZE"
done
# first-step variants (no residual yet) are not the steady-state step
python3 tools/pmc_all.py gpurun_out/r05_pmc_secondary.json --last 3 --exclude "threshold:<1>" --exclude "randomk:<false>" --exclude "dgc:spec_kernel<false>" --exclude "ddp_segmented:seg_main_kernel<false|seg_prep_kernel<false" --exclude "topk_sharded:topk_main<false|topk_bracket<false|stream_kernel" $args
