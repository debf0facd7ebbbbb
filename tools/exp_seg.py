"""Diagnostic: per-segment state of the segmented top-k after each step of the bench's ddp_segmented
scenario (ResNet-50 shapes, gradients rewritten in place by the step), read from the large segments'
workspaces: status (1 = exact fallback), n_sure, n_cand, need, boundary bin size, k, n."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from grace_amd.dist.segmented import SegmentedTopK  # noqa: E402
from grace_amd.harness import GradBucket, ShapeModel, step_segmented  # noqa: E402

dev = torch.device("cuda", 0)
model = ShapeModel(bench.resnet50_shapes(), dev)
bucket = GradBucket(model)
bucket.flat.normal_()
eng = SegmentedTopK(0.01)
sizes = bucket.sizes
for step in range(4):
    step_segmented(bucket, eng)
    torch.cuda.synchronize()
    for key, T in eng._tables.items():
        if key[3] != (step > 0):
            continue
        ws = T["ws"].cpu().numpy()
        offs = T["ws_off"].cpu().numpy()
        large = T["large"].cpu().numpy()[:T["n_large"]]
        rows = []
        for li, s in enumerate(large):
            c = ws[offs[li]:offs[li] + 64].view(np.uint32)
            n = sizes[s]
            k = max(1, int(n * 0.01))
            st = ws[offs[li] + 64:offs[li] + 256].view(np.uint64)
            us = lambda a, b: (int(st[b]) - int(st[a])) / 100.0   # noqa: E731
            rows.append((int(s), n, k, int(c[3]), int(c[4]), int(c[5]), int(c[9]), int(c[7]),
                         us(8, 9), us(9, 10), us(10, 11), us(11, 12), us(8, 12)))
        fb = [r for r in rows if r[3]]
        # absolute stamps relative to the first large segment's finalize start (slot 8, block 0)
        t0 = int(ws[offs[0] + 64:offs[0] + 256].view(np.uint64)[8])
        rel = []
        for li, s in enumerate(large):
            st = ws[offs[li] + 64:offs[li] + 256].view(np.uint64)
            rel.append((int(s), sizes[s], *[(int(st[q]) - t0) / 100.0 for q in (9, 10, 11, 12)]))
        rel.sort(key=lambda r: -r[5])
        print("  finalize stamps (us from the kernel start): seg n findB route last end; latest 6:")
        for r in rel[:6]:
            print("    seg %d n %d  %.1f %.1f %.1f %.1f" % r)
        # whole-step phases of the large segments, us from the earliest prep start (slot 13):
        # prep start / samples in / prep end (13, 14, 15), main span (16, 17), finalize start / end (8, 12)
        sts = [ws[offs[li] + 64:offs[li] + 256].view(np.uint64) for li in range(len(large))]
        p0 = min(int(x[13]) for x in sts)
        ph = lambda q: [(int(x[q]) - p0) / 100.0 for x in sts]   # noqa: E731
        for nm, q in (("prep_start", 13), ("prep_samples", 14), ("prep_end", 15), ("main_first", 16),
                      ("main_last", 17), ("fin_start", 8), ("fin_end", 12)):
            v = ph(q)
            print("  %-13s min %7.1f  median %7.1f  max %7.1f" % (nm, min(v), float(np.median(v)), max(v)))
        print(f"step {step}: {len(rows)} large segments, fallbacks {len(fb)}")
        slow = sorted(rows, key=lambda r: -r[-1])[:3]   # the slowest finalizes
        fix = [(int(large[li]), sizes[large[li]],
                int(ws[offs[li] + 64:offs[li] + 256].view(np.uint64)[18]),
                int(ws[offs[li] + 64:offs[li] + 256].view(np.uint64)[19]),
                int(ws[offs[li]:offs[li] + 64].view(np.uint32)[5]),
                int(ws[offs[li]:offs[li] + 64].view(np.uint32)[15]),
                int(ws[offs[li]:offs[li] + 64].view(np.uint32)[0]),
                int(ws[offs[li]:offs[li] + 64].view(np.uint32)[1])) for li in range(len(large))]
        print("  fix-up writes: total selected-below-mid %d, rejected-above-mid %d, candidates %d" %
              (sum(f[2] for f in fix), sum(f[3] for f in fix), sum(f[4] for f in fix)))
        for f in sorted(fix, key=lambda f: -(f[2] + f[3]))[:5]:
            print("    seg %d n %d sel<mid %d rej>mid %d n_cand %d mid %#x lo %#x hi %#x" % f)
        for r in sorted(rows, key=lambda r: -r[1])[:8] + fb[:8] + slow:
            print("  seg %d n %d k %d status %d n_sure %d n_cand %d need %d n_bnd %d | fin us: findB %.1f route %.1f "
                  "to_last %.1f bnd %.1f total %.1f" % r)
