#!/bin/bash
# PowerSGD configs[3] step (bench.py --workload powersgd): psgd_outer4 row bands of 4 (shipped) vs 2 / 1
# rows per workgroup (libgrace_hip_orow{2,1}.so: 8 / 4 KiB written per workgroup), alternating processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r05
: > gpurun_out/r05/ab_outer_rows.txt
for r in 1 2 3; do
  for v in base orow2 orow1; do
    lib=$PWD/grace_amd/lib/libgrace_hip.so; [ $v != base ] && lib=$PWD/grace_amd/lib/libgrace_hip_$v.so
    echo -n "$v run $r: " >> gpurun_out/r05/ab_outer_rows.txt
    GRACE_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --workload powersgd --steps 100 --no-cpu-baseline \
      2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" \
      >> gpurun_out/r05/ab_outer_rows.txt || exit 1
  done
done
