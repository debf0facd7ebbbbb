#!/bin/bash
# r02 PMC session (final build): FETCH_SIZE / WRITE_SIZE passes (one counter per run, each under
# its own kill timeout) for the headline top-k step and every secondary workload, then the per-step
# summaries bench.py reads (profiles/pmc_topk_main.json, profiles/r02_pmc_secondary.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -s KILL 90 "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "gpurun_out/$name.log"; exit $rc; fi; }
for c in FETCH_SIZE WRITE_SIZE; do
  run "pmc_head_$c" rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_r02b_topk_$c" -o pmc \
      -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline
done
python3 tools/pmc_summary.py gpurun_out/pmc_r02b_topk_FETCH_SIZE gpurun_out/pmc_r02b_topk_WRITE_SIZE \
    "topk_main<true" 67108864 1 gpurun_out/pmc_topk_main.json
args=""
for wl in ${PMC_WL:-qsgd terngrad powersgd sign256 natural cnat fp16 qsgd_step terngrad_step topk_nomem randomk threshold dgc sign_bits}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${wl}_$c" rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_r02b_${wl}_$c" -o pmc \
        -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline
  done
  args="$args $wl=gpurun_out/pmc_r02b_${wl}_FETCH_SIZE,gpurun_out/pmc_r02b_${wl}_WRITE_SIZE"
done
# steady state: each kernel's last 3 dispatches (the timed steps); first-step kernel variants and
# topk_nomem's four-call comparison path left out of the per-step sums
python3 tools/pmc_all.py gpurun_out/pmc_r02b_secondary.json --last 3 \
    --exclude 'topk_nomem:scatter_add_tag|FillOp|topk_main<false, 0|topk_finalize<0>' \
    --exclude 'randomk:randomk_pass_kernel<false>' --exclude 'threshold:thr_comp_stats_kernel<1>' $args
