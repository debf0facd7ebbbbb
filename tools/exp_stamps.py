"""Diagnostic: per-phase timings of the top-k bracket / finalize kernels from the -DGRACE_STAMPS
build, plus the step's selection counters.  Run on the GPU box:
    GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so python tools/exp_stamps.py
PATH=bench (default): the headline's world-1 Allgather(TopK 1 %, Residual).step on 64 Mi elements
with three rotating gradient sets (the bench's step: carried bracket, fused main, finalize);
PATH=plain: ops.topk_residual_step without the carry (the fresh two-read bracket).
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = int(os.environ.get("N", 64 * 1024 * 1024))
ratio = float(os.environ.get("RATIO", "0.01"))
path = os.environ.get("PATH_KIND", "bench")
k = int(os.environ.get("K", 0)) or ops.ratio_k(n, ratio)
res_only = os.environ.get("RES_ONLY", "0") == "1"   # the sharded / W > 1 local step: no dense output
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
names = ["thr_lo", "thr_hi", "shift", "status", "n_sure", "n_cand", "n_sel", "n_bnd", "B", "need"]
if path == "bench":
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    comm = Allgather(TopKCompressor(ratio), ResidualMemory(), 1)
    run = lambda it: comm.step(gs[it % 3], "b")   # noqa: E731
else:
    r = 0.1 * torch.randn(n, device=dev)
    out = None if res_only else torch.empty_like(gs[0])
    run = lambda it: ops.topk_residual_step(gs[it % 3], r, True, 1.0, 1.0, k, out=out)   # noqa: E731
rows = []
for it in range(12):
    o = run(it)
    torch.cuda.synchronize()
    del o
    ws = ops.topk_workspace(n, k, dev)
    ctl = ws[:256].cpu().numpy()
    u32 = ctl[:64].view(np.uint32)
    st = ctl[64:256].view(np.uint64)
    counters = dict(zip(names, u32[:10].tolist()))
    us = lambda a, b: (int(st[b]) - int(st[a])) / 100.0   # noqa: E731
    rows.append({"br_b0_load_zero": us(0, 1), "br_b0_flush": us(1, 2), "br_to_last": us(2, 3),
                 "br_last_coarse_fine": us(3, 4), "br_publish": us(4, 5), "br_total": us(0, 5),
                 "br_end_to_fin_start": us(5, 8),
                 "fin_b0_findB": us(8, 9), "fin_b0_route": us(9, 10), "fin_b0_to_last": us(10, 11),
                 "fin_last_bnd": us(11, 12), "fin_total": us(8, 12), "k": k, **counters})
keys = [q for q in rows[0] if q not in ("thr_lo", "thr_hi", "shift", "B")]
print(json.dumps({"lib": os.environ.get("GRACE_HIP_LIB", "default"), "path": path, "n": n, "res_only": res_only,
                  "median_of_steps_3_to_11": {q: round(statistics.median(r[q] for r in rows[3:]), 2) for q in keys}}))
