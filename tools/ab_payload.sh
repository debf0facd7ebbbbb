#!/bin/bash
# A/B the world > 1 payload kernels (sort, bounds, accumulate) between library builds: rocprofv3
# kernel stats of tools/exp_wn_local.py (W=8) per build.  usage: bash tools/ab_payload.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for L in "$@"; do
  i=$((i + 1))
  GRACE_HIP_LIB=$L W=${W:-8} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/ab_payload_$i -o run -- python3 tools/exp_wn_local.py > gpurun_out/ab_payload_$i.log 2>&1 || exit 1
  python3 - "$L" gpurun_out/ab_payload_$i <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].replace("void ", "").replace("grace::", ""): round(float(r["AverageNs"]) / 1e3, 1)
      for r in csv.DictReader(open(f)) if "grace" in r["Name"]}
print(sys.argv[1].split("/")[-1], {k: v for k, v in ks.items() if "group" in k or "chunk" in k or "finalize" in k})
PY
done
