"""Sharded top-k (grace_amd/dist/sharded.py + topk.hip "Sharded top-k") with the NATIVE kernels:
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


def _worker(rank, world, path, outdir, sizes, case, ratio, steps):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded import ShardedTopK
    n = sum(sizes)
    base = sum(sizes[:rank])
    eng = ShardedTopK(ratio)
    res = {}
    for s in range(steps):
        full = _bucket(case, n, 100 + s)
        out = eng.step(torch.from_numpy(full[base:base + sizes[rank]].copy()).cuda(), "bucket")
        v, i = eng.last_payload
        v, i = v.cpu().numpy(), i.cpu().numpy()
        keep = i >= 0
        res[f"out{s}"] = out.cpu().numpy()
        res[f"vals{s}"] = v[keep]
        res[f"idx{s}"] = i[keep]
        res[f"res{s}"] = eng.residuals["bucket"].cpu().numpy()
        res[f"fb{s}"] = np.array([eng.last_fallback])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("world,sizes,case,ratio", [
    (2, [1 << 20, 1 << 20], "normal", 0.01),
    (2, [(1 << 20) + 5, 777777], "normal", 0.001),
    (3, [300001, 300001, 300001], "normal", 0.01),
    (2, [400000, 400000], "ties", 0.5),
])
def test_sharded_topk_native_matches_single_gpu(world, sizes, case, ratio):
    from grace_amd import ops
    steps = 2
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
    assert not any(o[f"fb{s}"][0] for o in outs for s in range(steps))
