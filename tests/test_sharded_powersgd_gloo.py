"""Sharded PowerSGD (grace_amd/dist/sharded_powersgd.py) on CPU with gloo, W = 2 and 3.  The device
calls are replaced by torch CPU restatements (P = M q with the step's draws, the reference's modified
Gram-Schmidt, Q = Mᵀ P, P Qᵀ, the residual); the row partition, the P all-gather and the Q all-reduce
are the product's.  Expected: the oracle's whole-matrix PowerSGD (oracle.powersgd_compress /
powersgd_decode, powersgd.py:30-65) with the same q, within f32 tolerance (rel <= 1e-5·sqrt(m),
SURVEY §8a row a17), over two steps with error feedback (memory/powersgd.py:16-37).  The native GPU
version is tests/test_gpu_sharded_powersgd.py."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O

F32 = np.float32
N, M, NAME = 300, 160, "fc"


def _q(seed, m, r):
    g = torch.Generator().manual_seed(seed % (2 ** 63))
    return torch.randn(m, r, generator=g)


class OraclePowerSGDKernels:
    def p_draw(self, Mi, r, seed, out=None):
        P = Mi @ _q(seed, Mi.shape[1], r)
        if out is not None:
            out.copy_(P)
            return out
        return P

    def orthogonalize_(self, P):
        P.copy_(torch.from_numpy(O.orthogonalize(P.numpy())))
        return P

    def qt(self, Mi, P):
        return Mi.t() @ P

    def outer(self, P, Q, M=None):
        d = P @ Q.t()
        return d if M is None else M - d

    def add(self, a, b):
        return b + a


def _mat(step, n=N):
    return np.random.default_rng(300 + step).standard_normal((n, M)).astype(F32)


def _worker(rank, world, path, outdir, dense, n=N):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.sharded_powersgd import ShardedPowerSGD
    eng = ShardedPowerSGD(4, dense=dense, memory=True, kernels=OraclePowerSGDKernels())
    lo, hi = eng.partition(n, world)[rank]
    res = {}
    for s in range(2):
        res[f"out{s}"] = eng.step(torch.from_numpy(_mat(s, n)[lo:hi].copy()), NAME, n).numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _oracle(n=N):
    from grace_amd import ops
    outs, r = [], None
    for s in range(2):
        t = _mat(s, n) if r is None else (_mat(s, n) + r).astype(F32)
        q = _q(ops.step_seed("powersgd-q", NAME, s + 1), M, min(n, M, 4)).numpy()   # powersgd.py:36
        p, qq = O.powersgd_compress(t, q)
        d = O.powersgd_decode(p, qq)
        r = (t - d).astype(F32)
        outs.append(d)
    return outs


@pytest.mark.parametrize("world,n", [(2, N), (3, N), (3, 2)])
@pytest.mark.parametrize("dense", ["replicated", "shard"])
def test_sharded_powersgd_matches_oracle(world, n, dense):
    """(3, 2): a 2-row matrix over 3 ranks -- rank 2 holds no row, still joins the P all-gather and
    the Q all-reduce, and the rank is min(n, m, 4) = 2 (powersgd.py:36)."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, dense, n), nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    exp = _oracle(n)
    for s in range(2):
        got = [np.concatenate([o[f"out{s}"] for o in outs])] if dense == "shard" else [o[f"out{s}"] for o in outs]
        for g in got:
            assert np.abs(g - exp[s]).max() <= 1e-5 * np.sqrt(M) * np.abs(exp[s]).max(), s
