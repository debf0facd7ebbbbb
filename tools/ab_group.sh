set -o pipefail
mkdir -p gpurun_out/r05
for r in 1 2; do
  for v in base gp2 gp1 gb512; do
    if [ $v = base ]; then lib=grace_amd/lib/libgrace_hip.so; else lib=grace_amd/lib/libgrace_hip_$v.so; fi
    echo -n "$v $r: " >> gpurun_out/r05/ab_group.txt
    GRACE_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 tools/exp_wn_local.py >> gpurun_out/r05/ab_group.txt 2>&1 || exit 1
  done
done
