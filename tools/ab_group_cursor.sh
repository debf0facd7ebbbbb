#!/bin/bash
# Diagnostic: the grouping's scatter with its reservation atomics spread over 4 cursor copies
# (libgrace_hip_curcopies.so: WRONG positions, timing only) vs the shipped one -- how much of the
# scatter is the same-address chain of 164 workgroups' returning adds per chunk cursor.  (The build knob
# GRACE_DIAG_CURSOR_COPIES was removed after this A/B: no gain, profiles/r05_group2_ab.txt.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_group_cursor.txt
for r in 1 2 3; do
  for v in base curcopies; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v != base ] && lib=$PWD/grace_amd/lib/libgrace_hip_$v.so
    echo -n "$v $r: " >> gpurun_out/r05/ab_group_cursor.txt
    GRACE_HIP_LIB=$lib timeout -k 10 120 python3 tools/exp_wn_local.py 2>/dev/null >> gpurun_out/r05/ab_group_cursor.txt || exit 1
  done
done
