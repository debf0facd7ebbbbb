"""Sharded top-k protocol (grace_amd/dist/sharded.py) on CPU with gloo, W = 2 and 4.

The device calls (the local top-k + residual step and grace_shard_select) are replaced by an
oracle-backed numpy emulator that restates what each computes (grace_amd/csrc/shard.hip); the host
protocol, the one collective per step and the exactness argument are the product's.  Checked against the single-process oracle
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

HDR = 8


class OracleShardKernels:
    """numpy restatement of the sharded top-k device calls (test infrastructure): the local step is
    the oracle's single-bucket top-k + residual step (grace_topk_residual_step), the select
    restates grace_amd/csrc/shard.hip (exact cut over the gathered records by (|t| desc, global
    index asc), dense output 0 + v, own residual restored where the cut rejects a local pick)."""

    HDR = HDR

    def __init__(self):
        pass

    def record_words(self, cap):
        return HDR + 2 * cap

    def local_step(self, g, res, has_res, k_loc, vals, idx, res_out):
        t = O.residual_compensate(g.numpy().astype(np.float32), res.numpy() if has_res else None).ravel()
        v, i = O.topk_select(t, k_loc)
        r = t.copy()
        r[i] = t[i] - t[i]
        res_out.copy_(torch.from_numpy(r))
        vals[:k_loc] = torch.from_numpy(np.asarray(v, np.float32))
        idx[:k_loc] = torch.from_numpy(np.asarray(i, np.int64).astype(np.int32))

    def select(self, recs, world, rank, cap, tab, k, res, out, out_base, pay_idx, status):
        rv = recs.numpy().reshape(world, HDR + 2 * cap)
        tb = tab.numpy()
        sizes, bases = tb[:world], tb[world:]
        if any(int(rv[w, 0]) != int(sizes[w]) for w in range(world)):
            status[0] |= 1
        li = rv[:, HDR + cap:].astype(np.int64)
        v = rv[:, HDR:HDR + cap].copy().view(np.float32)
        gi = li + bases[:, None]
        valid = li >= 0
        keys = O.abs_key(v).astype(np.int64)
        flat = np.nonzero(valid.ravel())[0]
        order = np.lexsort((gi.ravel()[flat], -keys.ravel()[flat]))[:k]
        sel = np.zeros(world * cap, dtype=bool)
        sel[flat[order]] = True
        sel = sel.reshape(world, cap)
        o = out.numpy()
        q = gi[sel] - out_base
        ok = (q >= 0) & (q < o.size)
        o[q[ok]] = np.float32(0.0) + v[sel][ok]
        p = pay_idx.numpy()
        p[:] = np.where(sel[rank], gi[rank], -1).astype(np.int32)
        rej = valid[rank] & ~sel[rank]
        res.numpy()[li[rank][rej]] = v[rank][rej]

    def new_status(self, device):
        return torch.zeros(1, dtype=torch.int32)

    def take_status(self, st):
        bits = int(st[0])
        st[0] = 0
        return bits

    def fill_zero(self, x):
        return x.zero_()


def _bucket(case, n, seed):
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n).astype(np.float32)
    if case == "ties":       # 70 % zeros and k = 50 %: the k-th key is 0, a huge all-tie boundary bin
        g[rng.random(n) < 0.7] = 0.0
    if case == "miss":       # the even positions dominate
        g[::2] *= np.float32(1000.0)
    if case == "skew":       # the first quarter dominates: one rank holds the whole global top-k
        g[: n // 4] *= np.float32(100.0)
    return g


def _worker(rank, world, path, outdir, sizes, case, ratio, dense, sizes2=None, check_sizes=False, steps=2):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.sharded import ShardedTopK, ShardPartitionError
    eng = ShardedTopK(ratio, dense=dense, kernels=OracleShardKernels(), check_sizes=check_sizes)
    res = {}
    if steps > 2:    # step until one raises: record which (every rank must agree, nobody may hang)
        raised_at = -1
        for s in range(steps):
            part = sizes2 if (s >= 1 and sizes2 is not None) else sizes
            full = _bucket(case, sum(part), 100 + s)
            base = sum(part[:rank])
            try:
                eng.step(torch.from_numpy(full[base:base + part[rank]].copy()), "bucket")
            except ShardPartitionError:
                raised_at = s
                break
        np.savez(os.path.join(outdir, f"r{rank}.npz"), raised_at=np.array([raised_at]))
        dist.destroy_process_group()
        return
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
        res[f"rs{s}"] = np.array([eng.resizes])
    raised = 0
    try:
        eng.check(torch.device("cpu"))
    except ShardPartitionError:
        raised = 1
    res["raised"] = np.array([raised])
    res["host_reads"] = np.array([eng.host_reads])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _run(world, sizes, case, ratio, dense="replicated", sizes2=None, check_sizes=False, steps=2):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, sizes, case, ratio, dense, sizes2, check_sizes,
                                steps),
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
    (2, [150000, 150000], "miss", 0.01),             # the top-k sits on the even positions
    (3, [150000, 120001, 99999], "miss", 0.01),      # unequal shards
    (4, [30000, 30000, 30000, 30000], "skew", 0.01), # every selected entry on one rank
    (3, [500, 40000, 500], "normal", 0.01),          # shards shorter than k: short records
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
    # one host read (the partition, first step), none in the later step, nothing raised
    assert all(int(o["host_reads"][0]) == 1 and int(o["raised"][0]) == 0 for o in outs)


def test_sharded_resize_one_rank_between_steps():
    """ADVICE r1/r2, with check_sizes=True: only rank 1's shard changes size at step 2.  Every rank
    must see it in the same step (no rank-local collective, no hang) and re-plan with the new
    partition.  Rank 0's shard
    kept its size, so it keeps its error feedback (t = r + g, residual.py:10-14); rank 1 starts
    from t = g.  The event is counted in ``resizes`` on every rank."""
    sizes, sizes2 = [40000, 40000], [40000, 25000]
    outs = _run(2, sizes, "normal", 0.01, sizes2=sizes2, check_sizes=True)
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


def test_sharded_resize_without_check_sizes_is_reported():
    """Default mode (no per-step host read): a rank whose shard changes size after the first step
    cannot be seen by the others on the host, so the select kernels compare every record's shard
    length with the agreed partition and every rank raises ShardPartitionError afterwards -- the
    step neither hangs nor passes silently."""
    outs = _run(2, [40000, 40000], "normal", 0.01, sizes2=[40000, 25000])
    assert all(int(o["raised"][0]) == 1 for o in outs)


def test_sharded_resize_reported_at_the_same_step_on_every_rank():
    """without check(), the status of step N is taken at step N + 2 from a word only step
    N wrote (one per step parity), after step N's select has finished on that rank -- so every rank
    raises at the same step and none is left waiting in the next all-gather.  Rank 1's shard
    shrinks at step 1; both ranks raise at step 3."""
    outs = _run(2, [40000, 40000], "normal", 0.01, sizes2=[40000, 25000], steps=6)
    assert [int(o["raised_at"][0]) for o in outs] == [3, 3]
