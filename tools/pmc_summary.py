"""Per-launch HBM traffic of one kernel from two separate rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE), with the gfx950 corrections of MI355X_MICROARCH.md: FETCH_SIZE is in KB and counts
64-B requests as 32 B (x2), WRITE_SIZE is in KB.  Writes profiles/pmc_<name>.json for bench.py.
usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR NUMEL WORLD OUT_JSON"""
import collections
import csv
import json
import os
import sys


def per_launch(d, kernel):
    per = collections.defaultdict(float)
    with open(os.path.join(d, "pmc_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"]:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(per.values())


def main():
    fdir, wdir, kernel, numel, world, out = sys.argv[1:7]
    fetch = per_launch(fdir, kernel)
    write = per_launch(wdir, kernel)
    f_b = sum(fetch) / len(fetch) * 1024 * 2
    w_b = sum(write) / len(write) * 1024
    res = {"kernel": kernel, "numel": int(numel), "world": int(world), "launches": [len(fetch), len(write)],
           "fetch_bytes_per_launch": round(f_b), "write_bytes_per_launch": round(w_b),
           "hbm_bytes_per_launch": round(f_b + w_b),
           "source": [fdir, wdir], "correction": "FETCH_SIZE KB x1024 x2 (gfx950), WRITE_SIZE KB x1024"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
