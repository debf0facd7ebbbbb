"""Per-step HBM traffic of a workload's grace kernels from two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), with MI355X_MICROARCH.md's gfx950 corrections: FETCH_SIZE is in KB and a
wide (16-B per lane) streaming read is tallied at half its bytes (x2); WRITE_SIZE is in KB and
exact for 16-B-per-lane stores.  Other access widths (the codecs' 4-B code stores, 8-B loads) are
uncalibrated, so the per-kernel figures are reported raw-corrected and flagged.
usage: python tools/pmc_all.py OUT_JSON [--last N] [--exclude WL:REGEX] [--mode WL=MODE] WORKLOAD=FETCH_DIR,WRITE_DIR [...]"""
import collections
import csv
import json
import os
import sys


def per_kernel(d):
    """{kernel: [per-dispatch counter totals]} for the grace:: kernels of one pass."""
    disp = collections.defaultdict(float)
    name = {}
    path = None
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    if path is None:
        raise SystemExit(f"no counter_collection.csv under {d}")
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            if "grace::" not in k:
                continue
            disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = k.split("(")[0].replace("void ", "")
    out = collections.defaultdict(list)
    for did in sorted(disp, key=int):     # dispatch order, so `--last` keeps the timed steps
        out[name[did]].append(disp[did])
    return out


def main():
    """Options before the workloads: --last N averages only each kernel's last N dispatches (the
    timed steps; warm-up and first-step variants drop out), --exclude WL:REGEX leaves kernels whose
    name matches out of WL's per-step sum (e.g. a comparison path the bench also runs)."""
    import re
    res = {"correction": "FETCH_SIZE KB x1024 x2 (gfx950 16-B streaming reads), WRITE_SIZE KB x1024",
           "workloads": {}}
    args, last, excl, modes = sys.argv[2:], 0, {}, {}
    while args and args[0].startswith("--"):
        if args[0] == "--last":
            last = int(args[1])
        elif args[0] == "--exclude":
            w, rx = args[1].split(":", 1)
            excl[w] = re.compile(rx)
        elif args[0] == "--mode":   # WL=MODE: the output mode the passes ran in (bench.py checks it)
            w, m = args[1].split("=", 1)
            modes[w] = m
        args = args[2:]
    if last:
        res["steady_state"] = f"mean of each kernel's last {last} dispatches"
    for arg in args:
        wl, dirs = arg.split("=", 1)
        fdir, wdir = dirs.split(",")
        fk, wk = per_kernel(fdir), per_kernel(wdir)
        if last:
            fk = {k: v[-last:] for k, v in fk.items()}
            wk = {k: v[-last:] for k, v in wk.items()}
        if wl in excl:
            fk = {k: v for k, v in fk.items() if not excl[wl].search(k)}
            wk = {k: v for k, v in wk.items() if not excl[wl].search(k)}
        kern = {}
        step = 0.0
        for k in sorted(set(fk) | set(wk)):
            f = sum(fk.get(k, [0])) / max(len(fk.get(k, [])), 1) * 1024 * 2
            w = sum(wk.get(k, [0])) / max(len(wk.get(k, [])), 1) * 1024
            kern[k] = {"launches": [len(fk.get(k, [])), len(wk.get(k, []))], "fetch_bytes": round(f),
                       "write_bytes": round(w), "hbm_bytes": round(f + w)}
            step += f + w
        res["workloads"][wl] = {"kernels": kern, "hbm_bytes_per_step": round(step),
                                "source": [fdir, wdir]}
        if wl in modes:
            res["workloads"][wl]["mode"] = modes[wl]
    with open(sys.argv[1], "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({w: v["hbm_bytes_per_step"] for w, v in res["workloads"].items()}))


if __name__ == "__main__":
    main()
