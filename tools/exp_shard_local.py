"""Per-rank device time of the sharded top-k step (BASELINE configs[4]: 2^26 elements, k = 0.1 %,
W = 8) without the collective: one process plays every rank -- each rank's local top-k into its
slot of the gathered-records buffer (what the all-gather would deliver), then each rank's
grace_shard_select and its dense-output zero-fill -- timed with events per rank and phase, and
checked against the single-bucket oracle selection.  Usage: python tools/exp_shard_local.py [W]"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 1 << 26
ratio = 0.001
dev = torch.device("cuda", 0)
k = ops.ratio_k(n, ratio)
sizes = [n // W + (1 if r < n % W else 0) for r in range(W)]
bases = [sum(sizes[:r]) for r in range(W)]
cap = k
stride = ops.shard_record_words(cap)
tab = torch.tensor(sizes + bases, dtype=torch.int64, device=dev)
recs = torch.full((W * stride,), -1, dtype=torch.int32, device=dev)
for r in range(W):
    recs[r * stride] = sizes[r]
    recs[r * stride + 1:r * stride + ops.SHARD_HDR] = 0
gen = torch.Generator(device=dev)
gen.manual_seed(5)
g = torch.randn(n, device=dev, generator=gen)
res = [torch.zeros(sizes[r], device=dev) for r in range(W)]
res2 = [torch.zeros(sizes[r], device=dev) for r in range(W)]
pay = [torch.full((cap,), -1, dtype=torch.int32, device=dev) for r in range(W)]
st = ops.new_status_word()
ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
rows = []
for step in range(6):
    t_local, t_fill, t_sel = [], [], []
    for r in range(W):
        o = r * stride + ops.SHARD_HDR
        vals = recs[o:o + cap].view(torch.float32)
        idx = recs[o + cap:o + 2 * cap]
        a, b = ev(), ev()
        a.record()
        # (the product's local step: the new residual into a second buffer, ShardedTopK r05)
        ops.topk_residual_step_swap(g[bases[r]:bases[r] + sizes[r]], res[r], step > 0, 1.0, 1.0, min(cap, sizes[r]),
                                    res2[r], payload=(None, vals, idx))
        res[r], res2[r] = res2[r], res[r]
        b.record()
        t_local.append((a, b))
    outs = []
    for r in range(W):
        a, b, c = ev(), ev(), ev()
        a.record()
        out = torch.empty(n, device=dev)
        ops.fill(out, 0.0)
        b.record()
        ops.shard_select(recs, W, r, cap, tab, k, res[r], out, 0, pay[r], st)
        c.record()
        t_fill.append((a, b))
        t_sel.append((b, c))
        outs.append(out)
    torch.cuda.synchronize()
    ms = lambda pr: statistics.mean(x.elapsed_time(y) * 1e3 for x, y in pr)   # noqa: E731
    rows.append((ms(t_local), ms(t_fill), ms(t_sel)))
    if step == 0:   # exactness against the oracle's whole-bucket selection (first step, no residual)
        from oracle import grace_oracle as O
        gn = g.cpu().numpy()
        _, ii = O.topk_select(gn, k)
        got = np.sort(np.concatenate([p.cpu().numpy() for p in pay]))
        got = got[got >= 0]
        assert np.array_equal(got, np.sort(ii.astype(np.int64))), "selection differs from the oracle"
        o0 = outs[0].cpu().numpy()
        exp = np.zeros(n, np.float32)
        exp[ii] = np.float32(0.0) + gn[ii]
        assert np.array_equal(o0.view(np.uint32), exp.view(np.uint32)), "dense output differs"
    del outs
    if "stamps" in os.environ.get("GRACE_HIP_LIB", ""):   # the last rank's select, phase by phase
        ws = ops.workspace("shardsel", ops._lib.query("grace_shard_select_workspace_bytes", W, cap), dev)
        sv = ws[64:256].cpu().numpy().view(np.uint64)
        us = lambda a, b: round((int(sv[b]) - int(sv[a])) / 100.0, 1)   # noqa: E731
        nbv = ws[64 + 8 * 12:64 + 8 * 13].cpu().numpy().view(np.uint32)
        print(f"step {step} select stamps, us from the coarse launch's start (workgroup 0 unless noted): "
              f"coarse {us(0, 1)}, boundary {us(1, 2)}, apply {us(2, 3)}, boundary {us(3, 4)}, bnd to arrival "
              f"{us(4, 5)}, to the last arriver {us(5, 6)}, its ranking {us(6, 7)}; total {us(0, 7)}")
        print(f"  apply: find c1 {us(2, 8)}, round {us(8, 9)}, flush {us(9, 3)}; bnd: find b2 {us(4, 10)}, "
              f"rounds to arrival {us(10, 5)}; last arriver: load+pairwise {us(6, 13)}, decisions {us(13, 14)}, "
              f"re-zero {us(14, 7)}; nb {int(nbv[0])} n2 {int(nbv[1])}")
med = [statistics.median(r[i] for r in rows[2:]) for i in range(3)]
print(f"W={W} n={n} k={k} per-rank device time, us (median of steps 2..5): local top-k {med[0]:.1f}, "
      f"dense zero-fill {med[1]:.1f}, select {med[2]:.1f}; serial sum {sum(med):.1f} "
      f"(the fill runs on a side stream beside the local step and the exchange in ShardedTopK)")
print(f"oracle check: exact; status word {ops.status_take(st)}")
