#!/bin/bash
# The payload grouping without the histogram pass's tail (scatter workgroups scan the counts
# themselves) vs the r05 form (libgrace_hip_oldgroup.so): W = 8 per-rank step, alternating processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_group2.txt
for r in 1 2 3; do
  for v in new new1 oldgroup; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v != new ] && lib=$PWD/grace_amd/lib/libgrace_hip_$v.so
    echo -n "$v $r: " >> gpurun_out/r05/ab_group2.txt
    GRACE_HIP_LIB=$lib timeout -k 10 120 python3 tools/exp_wn_local.py 2>/dev/null >> gpurun_out/r05/ab_group2.txt || exit 1
  done
done
