"""Per-rank device time per step from a rocprofv3 --kernel-trace run of tools/exp_shard_codecs.py:
the grace:: kernels of each engine's dispatches (kernel_trace.csv, in dispatch order, split by the
engines' order in the run), divided by the rank-steps.  usage: python tools/shard_codecs_summary.py DIR W"""
import collections
import csv
import glob
import sys

d, W = sys.argv[1], int(sys.argv[2])
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
rows.sort()
# engines in run order; a kernel name belongs to the engine whose family it matches
fam = [("ShardedTernGrad", ("tern", "pack")), ("ShardedQuant(qsgd)", ("qsgd",)), ("ShardedPowerSGD", ("psgd", "powersgd", "orth", "normal"))]
steps = 12 * W   # 2 warm-up + 10 timed steps per rank
for name, keys in fam:
    per = collections.defaultdict(list)
    for a, b, k in rows:
        if "grace::" in k and any(x in k.lower() for x in keys):
            per[k].append((b - a) / 1e3)
    tot = 0.0
    print(f"{name}:")
    for k, v in sorted(per.items()):
        steady = v[len(v) * 2 // 12:]   # drop the warm-up share
        avg = sum(steady) / len(steady)
        calls = len(v) / steps
        tot += avg * calls
        print(f"  {k[:70]:70s} {calls:4.1f} per rank-step, avg {avg:7.2f} us")
    print(f"  per-rank device time per step (grace kernels, collective excluded): {tot:.1f} us")
