"""Summarise tools/pmc_sq.sh passes: per kernel (name substring of the grace kernels), the mean per
dispatch of every counter, the kernel-trace average duration, and derived figures (VALU busy share,
HBM bytes with the gfx950 FETCH_SIZE correction).  usage: python tools/pmc_sq_summary.py PREFIX"""
import collections
import csv
import glob
import json
import sys

prefix = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{prefix}_[0-9]*/**/pmc_counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, v in d.items():
            vals[k][c].append(v)
dur = {}
for f in glob.glob(f"{prefix}_kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"]) / 1e3
out = {}
for k, d in vals.items():
    if "grace" not in k:
        continue
    m = {c: sum(v[-3:]) / len(v[-3:]) for c, v in d.items()}   # steady state: the last 3 dispatches
    row = {c: round(v, 1) for c, v in m.items()}
    if "FETCH_SIZE" in m:
        row["hbm_read_MB"] = round(m["FETCH_SIZE"] * 2048 / 1e6, 2)
    if "WRITE_SIZE" in m:
        row["hbm_write_MB"] = round(m["WRITE_SIZE"] * 1024 / 1e6, 2)
    if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m and m.get("SQ_WAVE_CYCLES"):
        row["valu_share_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"], 3)
    if "SQ_WAIT_INST_ANY" in m and m.get("SQ_WAVE_CYCLES"):
        row["wait_share_of_wave_cycles"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    row["avg_us"] = next((v for n, v in dur.items() if n == k), None)
    out[k] = row
print(json.dumps(out, indent=1))
