#!/bin/bash
# Regression check of the bracket_search() refactor: the shipped library (main) vs one built from the
# topk.hip before it (libgrace_hip_preref.so): the headline step, alternating processes on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_preref.txt
for r in 1 2 3 4; do
  for v in main preref; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v != main ] && lib=$PWD/grace_amd/lib/libgrace_hip_$v.so
    echo -n "$v $r: " >> gpurun_out/r05/ab_preref.txt
    GRACE_HIP_LIB=$lib GRACE_BENCH_NO_PROBE=1 timeout -k 10 200 python3 bench.py --steps 40 --no-cpu-baseline \
      --no-overlap 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_us'])" \
      >> gpurun_out/r05/ab_preref.txt || exit 1
  done
done
