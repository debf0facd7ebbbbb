#!/bin/bash
# The bracket's search moved into the main pass (every main workgroup searches the sample histograms
# itself; the bracket ends after its flush -- a GRACE_MAIN_SEARCH=1 build as the main library) vs the bracket's last
# sampler searching (libgrace_hip_bsearch.so, GRACE_MAIN_SEARCH=0, shipped): the headline step, alternating
# processes on one box, ms per step (no in-bench probes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_main_search.txt
for r in 1 2 3 4; do
  for v in main bsearch; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v != main ] && lib=$PWD/grace_amd/lib/libgrace_hip_$v.so
    echo -n "$v $r: " >> gpurun_out/r05/ab_main_search.txt
    GRACE_HIP_LIB=$lib GRACE_BENCH_NO_PROBE=1 timeout -k 10 200 python3 bench.py --steps 40 --no-cpu-baseline \
      --no-overlap 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_us'])" \
      >> gpurun_out/r05/ab_main_search.txt || exit 1
  done
done
