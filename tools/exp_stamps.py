"""Diagnostic: per-phase timings of the top-k bracket / finalize kernels from the -DGRACE_STAMPS
build, plus the step's selection counters.  Run on the GPU box:
    GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so python tools/exp_stamps.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
ratio = float(os.environ.get("RATIO", "0.01"))
k = ops.ratio_k(n, ratio)
dev = torch.device("cuda", 0)
g = torch.randn(n, device=dev)
r = 0.1 * torch.randn(n, device=dev)
out = torch.empty_like(g)
rows = []
for it in range(8):
    ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    torch.cuda.synchronize()
    ws = ops.topk_workspace(n, k, dev)
    ctl = ws[:256].cpu().numpy()
    u32 = ctl[:64].view(np.uint32)
    st = ctl[64:256].view(np.uint64)
    names = ["thr_lo", "thr_hi", "shift", "status", "n_sure", "n_cand", "n_sel", "n_bnd", "B", "need"]
    counters = dict(zip(names, u32[:10].tolist()))
    us = lambda a, b: (int(st[b]) - int(st[a])) / 100.0
    rows.append({"smp_b0_load_zero": us(0, 1), "smp_b0_flush": us(1, 2), "smp_to_select": us(2, 3),
           "sel_copy": us(3, 4), "sel_find": us(4, 5), "br_total": us(0, 5),
           "fin_b0_findB": us(8, 9), "fin_b0_route": us(9, 10), "fin_b0_to_last": us(10, 11),
           "fin_last_bnd": us(11, 12), "fin_total": us(8, 12),
           "k": k, **counters})
import statistics  # noqa: E402
keys = [k for k in rows[0] if k not in ("thr_lo", "thr_hi", "shift", "B")]
print(os.environ.get("GRACE_HIP_LIB", "default"),
      {k: round(statistics.median(r[k] for r in rows[2:]), 2) for k in keys})
