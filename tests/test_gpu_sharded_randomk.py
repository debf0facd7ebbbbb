"""Sharded random-k + residual (grace_amd/dist/sharded_randomk.py) with the NATIVE kernels: 2 and 3
processes share cuda:0 over gloo.  Three steps of one name; every rank's result and residual shard
are compared bit-for-bit with the single-GPU ``Allgather(RandomKCompressor(ratio), ResidualMemory(),
1).step`` on the whole bucket (itself pinned against the reference in test_gpu_sparse.py), with the
device generator and with torch's CPU stream."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
F32 = np.float32
N, RATIO, NAME = (1 << 22) + 3, 0.01, "bucket0"


def _grad(step, n=N):
    return np.random.default_rng(90 + step).standard_normal(n).astype(F32)


def _worker(rank, world, path, outdir, dense, rng, n=N):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded_randomk import ShardedRandomK
    eng = ShardedRandomK(RATIO, dense=dense, rng=rng)
    lo, hi = eng.partition(n, world)[rank]
    res = {"lo": np.array([lo, hi])}
    for s in range(3):
        out = eng.step(torch.from_numpy(_grad(s, n)[lo:hi].copy()).cuda(), NAME, n)
        res[f"out{s}"] = out.cpu().numpy()
        res[f"res{s}"] = eng.residuals[NAME].cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _bits(a, b):
    return np.array_equal(np.asarray(a, F32).view(np.uint32), np.asarray(b, F32).view(np.uint32))


@pytest.mark.parametrize("world,n", [(2, N), (3, N), (3, 6)])
@pytest.mark.parametrize("dense,rng", [("replicated", "device"), ("shard", "device"), ("replicated", "torch_cpu")])
def test_sharded_randomk_native_matches_single_gpu(world, n, dense, rng):
    """(3, 6): 4-element blocks over 3 ranks, the last rank holds no element."""
    if n != N and rng == "torch_cpu":
        pytest.skip("the empty-rank case runs with the device generator")
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, dense, rng, n), nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    comm = Allgather(RandomKCompressor(RATIO, rng=rng), ResidualMemory(), 1)
    for s in range(3):
        exp = comm.step(torch.from_numpy(_grad(s, n)).cuda(), NAME).cpu().numpy()
        r = comm.memory.residuals[NAME].cpu().numpy()
        assert _bits(np.concatenate([o[f"res{s}"] for o in outs]), r), s
        if dense == "shard":
            assert _bits(np.concatenate([o[f"out{s}"] for o in outs]), exp), s
        else:
            for o in outs:
                assert _bits(o[f"out{s}"], exp), s
    if rng == "torch_cpu":
        # the torch-CPU stream is the reference's own: the reference restatement directly
        # (randomk.py:11-40 with ResidualMemory, residual.py:10-20), step by step
        from oracle import grace_oracle as O
        r = None
        for s in range(3):
            g = _grad(s, n)
            t = g if r is None else (r + g).astype(F32)
            idx, _ = O.randomk_indices(NAME, s, n, RATIO)
            d = O.randomk_decode(t[idx], idx, n)
            r = (t - d).astype(F32)
            assert _bits(np.concatenate([o[f"res{s}"] for o in outs]), r), (s, "residual vs oracle")
            out = (F32(0) + d).astype(F32)
            if dense == "replicated":
                for o in outs:
                    assert _bits(o[f"out{s}"], out), (s, "sharded vs oracle")
