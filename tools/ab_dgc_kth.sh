#!/bin/bash
# DGC world-1 step (bench.py --workload dgc): thr0 by the three-digit radix select
# (GRACE_DGC_SAMPLE_KTH=1, the default) vs the sample's full top-k (=0), alternating processes, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_dgc_kth.txt
for r in 1 2 3; do
  for k in 1 0; do
    echo -n "kth=$k run $r: " >> gpurun_out/r05/ab_dgc_kth.txt
    GRACE_DGC_SAMPLE_KTH=$k timeout -k 10 200 python3 bench.py --workload dgc --steps 40 --no-cpu-baseline \
      2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" \
      >> gpurun_out/r05/ab_dgc_kth.txt || exit 1
  done
done
