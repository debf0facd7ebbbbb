set -e
for L in grace_amd/lib/libgrace_hip_su1.so grace_amd/lib/libgrace_hip_su2.so grace_amd/lib/libgrace_hip.so grace_amd/lib/libgrace_hip_su8.so; do
  for st in 20 200; do
    r=$(GRACE_HIP_LIB=$L timeout -k 10 60 python3 bench.py --workload sign --steps $st | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
    echo "$L steps=$st ms=$r"
  done
done
