"""Sharded top-k protocol (grace_amd/dist/sharded.py) on CPU with gloo, W = 2 and 4.

The six device calls are replaced by an oracle-backed numpy emulator that restates what each HIP
kernel computes (grace_amd/csrc/topk.hip, "Sharded top-k"); the host protocol, the collectives
and the exactness argument are the product's.  Checked against the single-process oracle
top-k + residual step on the concatenated bucket: the union of the ranks' payloads is the same
set with the same values, every rank's residual shard is bit-identical, and the replicated dense
output is bit-identical.  The GPU version of this test is tests/test_gpu_sharded.py."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O

HIST = 2048
XCNT = 8
BRACKET_BINS = 32768


class OracleShardKernels:
    """numpy restatement of the sharded top-k kernels (test infrastructure)."""

    def __init__(self):
        self.state = {}

    def exchange_buffers(self, device):
        if "x" not in self.state:
            self.state["x"] = (torch.zeros(BRACKET_BINS, dtype=torch.int32), torch.zeros(HIST + XCNT, dtype=torch.int32))
        return self.state["x"]

    def empty(self, n, dtype, device):
        return torch.empty(n, dtype=dtype)

    def cand_cap(self, m, k):
        return min(m, 2 * k + 65536)

    @staticmethod
    def _t(g, res, has_res):
        gn = g.numpy().astype(np.float32)
        return O.residual_compensate(gn, res.numpy() if has_res else None).ravel()

    def sample(self, g, res, has_res, stratum, xs):
        t = self._t(g, res, has_res)
        sn = t.size // stratum
        pos = np.arange(sn, dtype=np.int64) * stratum + (stratum // 2)
        keys = O.abs_key(t[pos]) >> 16
        xs += torch.from_numpy(np.bincount(keys, minlength=BRACKET_BINS).astype(np.int32))

    def main(self, g, res, has_res, base, n, k, sample_total, vals, idx, xs, xh):
        # topk_select: global bracket from the all-reduced sample histogram
        h = xs.numpy().astype(np.int64)
        S = sample_total
        p = k / n
        mu = p * S
        sd = np.sqrt(mu * (1.0 - p) + 1.0)
        rank_hi = int(np.floor(mu - 6.0 * sd - 2.0))
        rank_lo = int(np.ceil(mu + 6.0 * sd + 2.0))
        r1 = [min(max(rank_hi, 0), S - 1) + 1, min(max(rank_lo, 0), S - 1) + 1]
        incl = np.cumsum(h[::-1])[::-1]            # count in bins >= b
        d = [int(np.nonzero(incl >= r)[0].max()) for r in r1]
        hi = (d[0] << 16) | 0xFFFF
        lo = d[1] << 16
        if rank_hi < 0:
            hi = 0x7FFFFFFF
        if rank_lo >= S:
            lo = 0
        lo = min(lo, hi)
        sh = 0
        while ((hi - lo) >> sh) >= HIST:
            sh += 1
        xs.zero_()
        xh.zero_()
        # topk_main, RES mode: r' = t everywhere, sure entries to the payload, candidates listed
        t = self._t(g, res, has_res)
        res.copy_(torch.from_numpy(t))
        key = O.abs_key(t).astype(np.int64)
        sure = np.nonzero(key > hi)[0]
        cand = np.nonzero((key <= hi) & (key >= lo))[0]
        ns = min(sure.size, k)
        vals[:ns] = torch.from_numpy(t[sure[:ns]])
        idx[:ns] = torch.from_numpy((sure[:ns] + base).astype(np.int32))
        bins = (key[cand] - lo) >> sh
        xh[:HIST] = torch.from_numpy(np.bincount(bins, minlength=HIST)[:HIST].astype(np.int32))
        xh[HIST] = sure.size
        xh[HIST + 1] = cand.size
        xh[HIST + 2] = t.size               # the shard length (sharded.py re-checks the partition)
        self.state.update(lo=lo, sh=sh, n_sure=ns, cand=cand, cand_t=t[cand], bins=bins, base=base)

    def route(self, res, base, k, B, vals, idx, bsend):
        st = self.state
        r = res.numpy()
        sel = idx[:st["n_sure"]].numpy().astype(np.int64) - base
        r[sel] = r[sel] - r[sel]
        above = st["bins"] > B
        a_i, a_t = st["cand"][above], st["cand_t"][above]
        p0 = st["n_sure"]
        vals[p0:p0 + a_i.size] = torch.from_numpy(a_t)
        idx[p0:p0 + a_i.size] = torch.from_numpy((a_i + base).astype(np.int32))
        r[a_i] = a_t - a_t
        st["n_pay"] = p0 + a_i.size
        inb = st["bins"] == B
        b_i, b_t = st["cand"][inb] + base, st["cand_t"][inb]
        bsend[0] = b_i.size
        packed = (b_i.astype(np.int64) & 0xFFFFFFFF) | (b_t.view(np.uint32).astype(np.int64) << 32)
        bsend[1:1 + b_i.size] = torch.from_numpy(packed)

    def boundary(self, res, base, k, brecv, world, cap_b, need, vals, idx, cap_p):
        st = self.state
        rv = brecv.numpy().reshape(world, cap_b + 1)
        ent = np.concatenate([rv[w, 1:1 + rv[w, 0]] for w in range(world)])
        gi = (ent & 0xFFFFFFFF).astype(np.int64)
        tv = (ent >> 32).astype(np.uint32).view(np.float32)
        order = np.lexsort((gi, -O.abs_key(tv).astype(np.int64)))[:need]
        r = res.numpy()
        m = r.size
        p = st["n_pay"]
        for j in sorted(order, key=lambda q: gi[q]):
            if base <= gi[j] < base + m:
                vals[p] = float(tv[j])
                idx[p] = int(gi[j])
                r[gi[j] - base] = tv[j] - tv[j]
                p += 1
        vals[p:cap_p] = 0.0
        idx[p:cap_p] = -1

    def take(self, vals_all, idx_all, k, res, base, vals, idx, cap_p):
        r = res.numpy()
        va, ia = vals_all.numpy(), idx_all.numpy().astype(np.int64)
        mine = (ia >= base) & (ia < base + r.size)
        c = int(mine.sum())
        vals[:c] = torch.from_numpy(va[mine])
        idx[:c] = torch.from_numpy(ia[mine].astype(np.int32))
        r[ia[mine] - base] = va[mine] - va[mine]
        vals[c:cap_p] = 0.0
        idx[c:cap_p] = -1

    def scatter_range(self, vals, idx, stride, per, world, base, out):
        o = out.numpy()
        for w in range(world):
            v = vals.numpy()[w * stride:w * stride + per]
            i = idx.numpy()[w * stride:w * stride + per].astype(np.int64)
            ok = (i >= base) & (i < base + o.size)
            o[i[ok] - base] = np.float32(0.0) + v[ok]

    def fill_zero(self, x):
        return x.zero_()

    def select_all(self, t, k):
        v, i = O.topk_select(t.numpy(), k)
        return torch.from_numpy(v), torch.from_numpy(i.astype(np.int32))


def _bucket(case, n, seed):
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n).astype(np.float32)
    if case == "ties":       # 70 % zeros and k = 50 %: the k-th key is 0, a huge all-tie boundary bin
        g[rng.random(n) < 0.7] = 0.0
    if case == "miss":       # the emulated sampler sees only odd positions; the even ones dominate
        g[::2] *= np.float32(1000.0)
    return g


def _worker(rank, world, path, outdir, sizes, case, ratio, dense, sizes2=None):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.sharded import ShardedTopK
    eng = ShardedTopK(ratio, dense=dense, kernels=OracleShardKernels())
    res = {}
    for s in range(2):
        part = sizes2 if (s == 1 and sizes2 is not None) else sizes
        n = sum(part)
        base = sum(part[:rank])
        full = _bucket(case, n, 100 + s)
        out = eng.step(torch.from_numpy(full[base:base + part[rank]].copy()), "bucket")
        v, i = eng.last_payload
        keep = i.numpy() >= 0
        res[f"out{s}"] = out.numpy().copy()
        res[f"vals{s}"] = v.numpy()[keep].copy()
        res[f"idx{s}"] = i.numpy()[keep].copy()
        res[f"res{s}"] = eng.residuals["bucket"].numpy().copy()
        res[f"fb{s}"] = np.array([eng.last_fallback])
        res[f"rs{s}"] = np.array([eng.resizes])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _run(world, sizes, case, ratio, dense="replicated", sizes2=None):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, sizes, case, ratio, dense, sizes2),
                 nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    return outs


def _bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("world,sizes,case,ratio", [
    (2, [40000, 40000], "normal", 0.01),
    (4, [30000, 30000, 30000, 30000], "normal", 0.01),
    (2, [50000, 33333], "normal", 0.01),
    (2, [40000, 40000], "ties", 0.5),
    (2, [150000, 150000], "miss", 0.01),
    (3, [150000, 120001, 99999], "miss", 0.01),      # fallback gather with unequal shards
])
def test_sharded_topk_matches_single_bucket(world, sizes, case, ratio):
    outs = _run(world, sizes, case, ratio)
    n = sum(sizes)
    r = None
    for s in range(2):
        g = _bucket(case, n, 100 + s)
        _, v, i, r_new, out = O.topk_residual_step(g, r, ratio)
        r = r_new
        idx = np.concatenate([o[f"idx{s}"] for o in outs]).astype(np.int64)
        vals = np.concatenate([o[f"vals{s}"] for o in outs])
        order = np.argsort(idx)
        assert np.array_equal(idx[order], i.astype(np.int64)), (s, world, case)
        assert _bits(vals[order], v)
        assert _bits(np.concatenate([o[f"res{s}"] for o in outs]), r_new)
        for o in outs:
            assert _bits(o[f"out{s}"], out)
    if case == "miss":       # bracket missed -> exact gather-and-select fallback
        assert all(o["fb0"][0] for o in outs)
    else:
        assert not any(o["fb0"][0] or o["fb1"][0] for o in outs)


def test_sharded_resize_one_rank_between_steps():
    """only rank 1's shard changes size at step 2.  Every rank must see it in the same
    step (no rank-local collective, no hang) and re-plan with the new partition.  Rank 0's shard
    kept its size, so it keeps its error feedback (t = r + g, residual.py:10-14); rank 1 starts
    from t = g.  The event is counted in ``resizes`` on every rank."""
    sizes, sizes2 = [40000, 40000], [40000, 25000]
    outs = _run(2, sizes, "normal", 0.01, sizes2=sizes2)
    g0 = _bucket("normal", sum(sizes), 100)
    _, _, i0, r0, out0 = O.topk_residual_step(g0, None, 0.01)
    idx = np.sort(np.concatenate([o["idx0"] for o in outs]).astype(np.int64))
    assert np.array_equal(idx, i0.astype(np.int64))
    g1 = _bucket("normal", sum(sizes2), 101)
    carried = np.concatenate([r0[:40000], np.zeros(25000, np.float32)])   # rank 0's residual kept
    _, v1, i1, r1, out1 = O.topk_residual_step(g1, carried, 0.01)
    idx = np.concatenate([o["idx1"] for o in outs]).astype(np.int64)
    vals = np.concatenate([o["vals1"] for o in outs])
    order = np.argsort(idx)
    assert np.array_equal(idx[order], i1.astype(np.int64))
    assert _bits(vals[order], v1)
    assert _bits(np.concatenate([o["res1"] for o in outs]), r1)
    for o in outs:
        assert _bits(o["out1"], out1)
        assert int(o["rs0"][0]) == 0 and int(o["rs1"][0]) == 1


def test_sharded_dense_shard_mode():
    sizes = [40000, 40000]
    outs = _run(2, sizes, "normal", 0.01, dense="shard")
    g = _bucket("normal", sum(sizes), 100)
    _, _, _, _, out = O.topk_residual_step(g, None, 0.01)
    assert _bits(np.concatenate([o["out0"] for o in outs]), out)


def test_plan_boundary_edge_cases():
    from grace_amd.dist.sharded import plan_boundary
    xh = np.zeros((2, HIST + XCNT), dtype=np.int64)
    xh[:, HIST] = [3, 2]                     # n_sure = 5
    xh[0, 10] = 4
    xh[1, 10] = 1
    xh[1, 7] = 6
    xh[:, HIST + 1] = xh[:, :HIST].sum(axis=1)   # n_cand
    assert plan_boundary(xh, 5, 2, 1000) == (True, HIST, 0, 0, 3)        # nothing else needed
    ok, B, need, cap_b, cap_p = plan_boundary(xh, 8, 2, 1000)            # 3 more: from bin 10
    assert (ok, B, need, cap_b) == (True, 10, 3, 4) and cap_p == 7
    ok, B, need, cap_b, cap_p = plan_boundary(xh, 12, 2, 1000)           # 7 more: bin 10 (5) + 2 of bin 7
    assert (ok, B, need, cap_b) == (True, 7, 2, 6)
    assert plan_boundary(xh, 4, 2, 1000)[0] is False                     # more sure than k
    assert plan_boundary(xh, 100, 2, 1000)[0] is False                   # too few candidates
