"""Steady-state per-kernel summary of a rocprofv3 --kernel-trace run of bench.py.

Reads <dir>/run_kernel_trace.csv, keeps the grace_amd kernels, and for each kernel name reports the
LAST `--last` launches only (the timed steps: warm-up and first steps dropped), plus the per-step
composition of the top-k step (bracket start -> finalize end, and the gaps between its kernels).
Usage: python tools/prof_steady.py gpurun_out/prof_r04_topk [--last 20] [--out profiles/x.json]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--out")
    args = ap.parse_args()
    rows = []
    with open(f"{args.dir}/run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "grace::" not in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    rows.sort()
    by = {}
    for s, e, n in rows:
        by.setdefault(n, []).append((s, e))
    summary = {}
    for n, v in by.items():
        d = [(e - s) / 1e3 for s, e in v[-args.last:]]
        summary[n] = {"launches_total": len(v), "launches_used": len(d), "avg_us": round(statistics.mean(d), 2),
                      "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                      "stdev_us": round(statistics.pstdev(d), 2)}
    # step composition: each bracket<true> opens a step; the step ends at the next finalize's end
    steps = []
    seq = [(s, e, n) for s, e, n in rows if n.startswith("grace::topk_")]
    for i, (s, e, n) in enumerate(seq):
        if n == "grace::topk_bracket<true>" and i + 2 < len(seq):
            (s1, e1, n1), (s2, e2, n2) = seq[i + 1], seq[i + 2]
            if n1.startswith("grace::topk_main") and n2.startswith("grace::topk_finalize"):
                steps.append({"bracket": (e - s) / 1e3, "gap1": (s1 - e) / 1e3, "main": (e1 - s1) / 1e3,
                              "gap2": (s2 - e1) / 1e3, "finalize": (e2 - s2) / 1e3, "span": (e2 - s) / 1e3})
    steps = steps[-args.last:]
    comp = {k: round(statistics.mean(st[k] for st in steps), 2) for k in steps[0]} if steps else {}
    out = {"source": args.dir, "note": f"last {args.last} launches per kernel (the timed steps); "
           "step = topk_bracket<true> start -> topk_finalize end", "kernels": summary,
           "step_composition_us": comp, "steps_used": len(steps)}
    txt = json.dumps(out, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
