#!/bin/bash
# rocprofv3 kernel-trace stats of one bench workload: tools/prof_one.sh WORKLOAD TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=$1; tag=$2; shift 2
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_${tag}" -o run \
  -- python3 bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu-baseline "$@" > "gpurun_out/prof_${tag}.log" 2>&1
rc=$?
f=$(find "gpurun_out/prof_${tag}" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-160
exit $rc
