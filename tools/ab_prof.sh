#!/bin/bash
# Per-kernel rocprofv3 averages of one bench workload across library variants, each in its own
# process: tools/ab_prof.sh WORKLOAD STEPS LIB [LIB ...]  -> gpurun_out/abprof_<workload>_<lib>/
# (kernel_stats.csv per variant) and one summary line per variant on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
wl=$1; st=$2; shift 2
for L in "$@"; do
  tag=$(basename "$L" .so)
  out=gpurun_out/abprof_${wl}_${tag}
  GRACE_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
      -- python3 bench.py --workload "$wl" --steps "$st" --warmup 5 --no-cpu-baseline > "$out.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -3 "$out.log"; exit $rc; fi
  python3 - "$out" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
rows = [r for r in rows if "grace" not in r["Name"].lower() or True]
top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:6]
print(sys.argv[2], " | ".join(f"{r['Name'].split('(')[0][:40]} {float(r['AverageNs'])/1e3:.2f}us x{r['Calls']}" for r in top))
PY
done
