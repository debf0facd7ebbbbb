#!/bin/bash
# DGC world-1 step: the shipped library vs a diagnostic build that skips the five gated fix-up
# launches (libgrace_hip_nofix.so, GRACE_DGC_NO_FIXUP): the cost of the no-op launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_dgc_fix.txt
for r in 1 2 3; do
  for v in base nofix; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v = nofix ] && lib=$PWD/grace_amd/lib/libgrace_hip_nofix.so
    echo -n "$v run $r: " >> gpurun_out/r05/ab_dgc_fix.txt
    GRACE_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --workload dgc --steps 40 --no-cpu-baseline \
      2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" \
      >> gpurun_out/r05/ab_dgc_fix.txt || exit 1
  done
done
