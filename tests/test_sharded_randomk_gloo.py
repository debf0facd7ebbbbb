"""Sharded random-k + residual (grace_amd/dist/sharded_randomk.py) on CPU with gloo, W = 2 and 3.
The device calls are replaced by a numpy restatement of what each computes (t = r + g, r' = t with
the drawn positions t - t, the owner's payload values, the 0 + v decode); the indices come from
torch's CPU stream (rng="torch_cpu"), as the reference draws them (randomk.py:26-30).  Three steps of
one name: every rank's residual shard and result must equal the oracle's whole-bucket sequence
(oracle.randomk_indices / residual_compensate / sparse decode, randomk.py:6-41, residual.py:10-20,
allgather.py:40-45).  The native GPU version is tests/test_gpu_sharded_randomk.py."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O

F32 = np.float32
N, RATIO, NAME = 10007, 0.05, "layer.weight"


class OracleRandomKKernels:
    def indices(self, h, n, k, rng, device):
        assert rng == "torch_cpu"
        return torch.randint(n, [k])

    def shard_step(self, g, res, has, beta, gamma, lo, idx, out):
        gv, m = g.numpy(), g.numel()
        t = O.residual_compensate(gv, res.numpy()) if has else gv.copy()
        i = idx.numpy() - lo
        own = (i >= 0) & (i < m)
        vals = np.where(own, t[np.clip(i, 0, m - 1)], F32(0)).astype(F32)
        r = t.copy()
        r[i[own]] = (t[i[own]] - t[i[own]]).astype(F32)
        res.copy_(torch.from_numpy(r))
        if out is not None:
            o = np.zeros(m, F32)
            o[i[own]] = (F32(0) + t[i[own]]).astype(F32)
            out.copy_(torch.from_numpy(o))
        return torch.from_numpy(vals)

    def decode(self, vals, idx, n):
        o = np.zeros(n, F32)
        o[idx.numpy()] = (F32(0) + vals.numpy()).astype(F32)
        return torch.from_numpy(o)


def _grad(step, n=N):
    return np.random.default_rng(50 + step).standard_normal(n).astype(F32)


def _worker(rank, world, path, outdir, dense, n=N):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.sharded_randomk import ShardedRandomK
    eng = ShardedRandomK(RATIO, dense=dense, rng="torch_cpu", kernels=OracleRandomKKernels())
    lo, hi = eng.partition(n, world)[rank]
    res = {}
    for s in range(3):
        out = eng.step(torch.from_numpy(_grad(s, n)[lo:hi].copy()), NAME, n)
        res[f"out{s}"] = out.numpy()
        res[f"res{s}"] = eng.residuals[NAME].numpy().copy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), lo=np.array([lo, hi]), **res)
    dist.destroy_process_group()


def _oracle(n=N):
    r = None
    outs, ress = [], []
    for s in range(3):
        g = _grad(s, n)
        t = g.copy() if r is None else O.residual_compensate(g, r)
        idx, _ = O.randomk_indices(NAME, s, n, RATIO)
        dec = O.randomk_decode(t[idx], idx, n)
        r = O.residual_update(t, dec)
        outs.append(O.python_sum([dec]))
        ress.append(r)
    return outs, ress


def _bits(a, b):
    return np.array_equal(np.asarray(a, F32).view(np.uint32), np.asarray(b, F32).view(np.uint32))


@pytest.mark.parametrize("world,n", [(2, N), (3, N), (3, 6)])
@pytest.mark.parametrize("dense", ["replicated", "shard"])
def test_sharded_randomk_matches_oracle_sequence(world, n, dense):
    """(3, 6): 4-element blocks over 3 ranks -- the last rank holds no element and still joins the
    all-reduce (replicated) or returns an empty slice (shard)."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, dense, n), nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    exp_out, exp_res = _oracle(n)
    for s in range(3):
        assert _bits(np.concatenate([o[f"res{s}"] for o in outs]), exp_res[s]), s
        if dense == "shard":
            assert _bits(np.concatenate([o[f"out{s}"] for o in outs]), exp_out[s]), s
        else:
            for o in outs:
                assert _bits(o[f"out{s}"], exp_out[s]), s
    assert outs[0]["lo"][0] == 0 and outs[-1]["lo"][1] == n
