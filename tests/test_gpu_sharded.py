"""Sharded top-k (grace_amd/dist/sharded.py + csrc/shard.hip) with the NATIVE kernels:
2 (and 3) processes share cuda:0 over gloo (RCCL needs one device per rank; the 8-GPU RCCL run is
the driver's).  The union of the ranks' payloads, their residual shards and the replicated dense
output are compared bit-for-bit with the single-GPU fused top-k + residual step on the whole
bucket (itself parity-tested against the oracle in test_gpu_topk.py), and with the oracle."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O

pytestmark = pytest.mark.gpu


def _bucket(case, n, seed):
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n).astype(np.float32)
    if case == "ties":
        g[rng.random(n) < 0.7] = 0.0
    return g


def _worker(rank, world, path, outdir, sizes, case, ratio, steps, dense="replicated"):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded import ShardedTopK
    n = sum(sizes)
    base = sum(sizes[:rank])
    eng = ShardedTopK(ratio, dense=dense)
    res = {}
    for s in range(steps):
        full = _bucket(case, n, 100 + s)
        # the result is dropped right away (as the DDP loop does): the next step recycles it and
        # zeroes only the previous selection (grace_shard_clear) instead of zero-filling all of it
        res[f"out{s}"] = eng.step(torch.from_numpy(full[base:base + sizes[rank]].copy()).cuda(), "bucket").cpu().numpy()
        v, i = eng.last_payload
        v, i = v.cpu().numpy(), i.cpu().numpy()
        keep = i >= 0
        res[f"vals{s}"] = v[keep]
        res[f"idx{s}"] = i[keep]
        res[f"res{s}"] = eng.residuals["bucket"].cpu().numpy()
    res["host_reads"] = np.array([eng.host_reads])
    res["recycled"] = np.array([eng._recycler.hits])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("world,sizes,case,ratio", [
    (2, [1 << 20, 1 << 20], "normal", 0.01),
    (2, [(1 << 20) + 5, 777777], "normal", 0.001),
    (3, [300001, 300001, 300001], "normal", 0.01),
    (2, [400000, 400000], "ties", 0.5),
    (2, [1 << 22, (1 << 22) - 3], "normal", 0.3),   # W * cap > 4 Mi entries: the three-launch select
])
def test_sharded_topk_native_matches_single_gpu(world, sizes, case, ratio):
    from grace_amd import ops
    steps = 3
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, sizes, case, ratio, steps),
                 nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    n = sum(sizes)
    k = ops.ratio_k(n, ratio)
    res_gpu = torch.empty(n, device="cuda")
    r_or = None
    for s in range(steps):
        g = _bucket(case, n, 100 + s)
        # single-GPU fused engine on the whole bucket
        out1 = torch.empty(n, device="cuda")
        _, vals1, idx1 = ops.topk_residual_step(torch.from_numpy(g).cuda(), res_gpu, s > 0, 1.0, 1.0, k, out=out1)
        # oracle
        _, v_or, i_or, r_or, out_or = O.topk_residual_step(g, r_or, ratio)
        idx = np.concatenate([o[f"idx{s}"] for o in outs]).astype(np.int64)
        vals = np.concatenate([o[f"vals{s}"] for o in outs])
        order = np.argsort(idx)
        assert np.array_equal(idx[order], i_or.astype(np.int64)), (s, world, case)
        assert _bits(vals[order], v_or)
        i1 = idx1.cpu().numpy().astype(np.int64)
        assert np.array_equal(np.sort(i1), idx[order])
        r_cat = np.concatenate([o[f"res{s}"] for o in outs])
        assert _bits(r_cat, r_or)
        assert _bits(r_cat, res_gpu.cpu().numpy())
        for o in outs:
            assert _bits(o[f"out{s}"], out_or)
        assert _bits(outs[0][f"out{s}"], out1.cpu().numpy())
    # the partition is agreed once (first step); the later steps read nothing on the host
    assert all(int(o["host_reads"][0]) == (1 if world > 1 else 0) for o in outs)
    # every step after the first reused its dropped output
    assert all(int(o["recycled"][0]) == steps - 1 for o in outs)


def _resize_worker(rank, world, path, outdir, check_sizes):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded import ShardedTopK, ShardPartitionError
    eng = ShardedTopK(0.01, check_sizes=check_sizes)
    res = {}
    for s, sizes in enumerate(([300000, 300000], [300000, 200000])):
        base = sum(sizes[:rank])
        full = _bucket("normal", sum(sizes), 100 + s)
        out = eng.step(torch.from_numpy(full[base:base + sizes[rank]].copy()).cuda(), "bucket")
        v, i = eng.last_payload
        v, i = v.cpu().numpy(), i.cpu().numpy()
        res[f"out{s}"] = out.cpu().numpy()
        res[f"vals{s}"] = v[i >= 0]
        res[f"idx{s}"] = i[i >= 0]
        res[f"res{s}"] = eng.residuals["bucket"].cpu().numpy()
    raised = 0
    try:
        eng.check()
    except ShardPartitionError:
        raised = 1
    res["raised"] = np.array([raised, eng.resizes])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("check_sizes", [True, False])
def test_sharded_resize_native(check_sizes):
    """Rank 1's shard shrinks at step 2.  check_sizes=True: every rank re-plans in that step, the
    result equals the single-bucket oracle with rank 0's error feedback kept and rank 1 starting
    from t = g.  Default: no per-step host read, and the mixed partition is reported on every rank
    (ShardPartitionError from check()) instead of hanging or passing silently."""
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_resize_worker, args=(world, os.path.join(tmp, "rdv"), tmp, check_sizes), nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    g0 = _bucket("normal", 600000, 100)
    _, _, i0, r0, out0 = O.topk_residual_step(g0, None, 0.01)
    idx = np.sort(np.concatenate([o["idx0"] for o in outs]).astype(np.int64))
    assert np.array_equal(idx, i0.astype(np.int64))
    for o in outs:
        assert _bits(o["out0"], out0)
    if not check_sizes:
        assert all(int(o["raised"][0]) == 1 for o in outs)
        return
    g1 = _bucket("normal", 500000, 101)
    carried = np.concatenate([r0[:300000], np.zeros(200000, np.float32)])   # rank 0's residual kept
    _, v1, i1, r1, out1 = O.topk_residual_step(g1, carried, 0.01)
    idx = np.concatenate([o["idx1"] for o in outs]).astype(np.int64)
    vals = np.concatenate([o["vals1"] for o in outs])
    order = np.argsort(idx)
    assert np.array_equal(idx[order], i1.astype(np.int64))
    assert _bits(vals[order], v1)
    assert _bits(np.concatenate([o["res1"] for o in outs]), r1)
    for o in outs:
        assert _bits(o["out1"], out1)
        assert int(o["raised"][0]) == 0 and int(o["raised"][1]) == 1


@pytest.mark.parametrize("world,sizes,case,ratio", [
    (2, [1 << 20, 1 << 20], "normal", 0.01),
    (2, [(1 << 20) + 5, 777777], "ties", 0.3),
])
def test_sharded_topk_native_dense_shard(world, sizes, case, ratio):
    """SURVEY §8e's sharded-decode mode (dense="shard") with the native kernels:
    every rank's output is exactly its own slice of the single-bucket decoded result (bit-exact
    against the oracle), over three steps with recycled outputs; payloads and residuals as the
    replicated mode."""
    steps = 3
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, sizes, case, ratio, steps, "shard"),
                 nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    n = sum(sizes)
    r_or = None
    for s in range(steps):
        g = _bucket(case, n, 100 + s)
        _, v_or, i_or, r_or, out_or = O.topk_residual_step(g, r_or, ratio)
        idx = np.concatenate([o[f"idx{s}"] for o in outs]).astype(np.int64)
        vals = np.concatenate([o[f"vals{s}"] for o in outs])
        order = np.argsort(idx)
        assert np.array_equal(idx[order], i_or.astype(np.int64)), s
        assert _bits(vals[order], v_or)
        assert _bits(np.concatenate([o[f"res{s}"] for o in outs]), r_or)
        for w, o in enumerate(outs):
            assert o[f"out{s}"].size == sizes[w]
        assert _bits(np.concatenate([o[f"out{s}"] for o in outs]), out_or), s
    assert all(int(o["recycled"][0]) == steps - 1 for o in outs)


def _raise_worker(rank, world, path, outdir):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded import ShardedTopK, ShardPartitionError
    eng = ShardedTopK(0.01)
    raised_at = -1
    for s in range(6):
        sizes = [300000, 300000] if s == 0 else [300000, 200000]
        base = sum(sizes[:rank])
        full = _bucket("normal", sum(sizes), 100 + s)
        try:
            eng.step(torch.from_numpy(full[base:base + sizes[rank]].copy()).cuda(), "bucket")
        except ShardPartitionError:
            raised_at = s
            break
    np.savez(os.path.join(outdir, f"r{rank}.npz"), raised_at=np.array([raised_at]))
    dist.destroy_process_group()


def test_sharded_resize_raised_by_step_on_every_rank():
    """with no check() call, a resize at step 1 is raised by step() itself, at the same
    step on both ranks (step N's status word is taken at step N + 2 after step N's select event),
    so neither rank is left blocked in the next all-gather."""
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_raise_worker, args=(world, os.path.join(tmp, "rdv"), tmp), nprocs=world, join=True)
        got = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                got.append(int(z["raised_at"][0]))
    assert got == [3, 3]
