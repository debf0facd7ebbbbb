"""Per-step kernel durations and launch gaps of the top-k step from a rocprofv3 kernel trace.
usage: python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [name-substring]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "grace::topk"
rows = [r for r in rows if sub in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    dur[name].append((e - s) / 1e3)
    if prev is not None:
        g = (s - prev[1]) / 1e3
        if g < 50:   # same burst of steps
            gap[prev[0] + " -> " + name].append(g)
    prev = (name, e)
for k, v in dur.items():
    print(f"{k:50s} n={len(v):4d} median {statistics.median(v):8.2f} us")
for k, v in gap.items():
    print(f"gap {k:70s} n={len(v):4d} median {statistics.median(v):6.2f} us")
