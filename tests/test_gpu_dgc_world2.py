"""DGC at world size 2 on one GPU (two processes share cuda:0 over gloo), through
``Allgather(DgcCompressor, DgcMemory, 2).step`` -- the variable-size exchange of SURVEY.md §8f.1 --
in every exchange mode of grace_amd/dist/compressor/dgc.py:

* ``exchange="counts"``: one host read of the W device counts per step;
* ``exchange="capacity", overflow="retry"``: fixed-size records, one stat read per step, an
  overflowing step redone through the counts exchange -- always the reference's result;
* ``exchange="capacity", overflow="defer"``: nothing read on the host in the common step; on
  overflow the first ``cap`` entries (index order) travel and the rest stay in the momentum memory.

Expected values come from the oracle (grace_dl/dist/compressor/dgc.py:12-50, memory/dgc.py:15-39,
communicator/allgather.py:15-45), with the reference's own sampling stream: every rank seeds torch's
CPU generator and DgcCompressor(rng="torch_cpu") draws ``uniform_(0, numel).long()`` from it as the
reference does, which the test replays.  The capacity bookkeeping (margin, growth on overflow,
shrink when 4x too large) is restated from dgc.py and checked step by step: bit-exact outputs,
residuals and accumulators on both ranks, and the same overflow count on both ranks.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
F32 = np.float32
N, RATIO, MOM, STEPS, W = 50_000, 0.01, 0.9, 6, 2


def _grad(rank, step):
    rng = np.random.default_rng(4000 + 10 * rank + step)
    g = rng.standard_normal(N, dtype=F32)
    if step == 3 and rank == 1:          # a heavier tail on one rank: more entries pass the threshold
        g[: N // 3] *= F32(6.0)
    return g


def _worker(rank, path, outdir, mode):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=W)
    torch.cuda.set_device(0)
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.dgc import DgcCompressor
    from grace_amd.dist.memory.dgc import DgcMemory
    exchange, margin, overflow = mode
    torch.manual_seed(1000 + rank)
    comp = DgcCompressor(RATIO, rng="torch_cpu", exchange=exchange, capacity_margin=margin, overflow=overflow)
    comm = Allgather(comp, DgcMemory(MOM, False, W), W)
    res = {}
    for s in range(STEPS):
        out = comm.step(torch.from_numpy(_grad(rank, s)).cuda(), "w")
        res[f"out{s}"] = out.cpu().numpy()
        res[f"r{s}"] = comm.memory.residuals["w"].cpu().numpy()
        res[f"a{s}"] = comm.memory.gradients["w"].cpu().numpy()
        res[f"cap{s}"] = np.array([comp.capacity.get("w", -1)])
    res["overflows"] = np.array([comp.overflows])
    res["host_reads"] = np.array([comp.host_reads])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _grow(mx, margin):
    return int(min(N, max(64, int(np.ceil(mx * margin)))))


def _expected(mode):
    """The reference's step, with the capacity policy of dgc.py restated."""
    exchange, margin, overflow = mode
    gens = []
    for r in range(W):
        gen = torch.Generator().manual_seed(1000 + r)
        gens.append(gen)
    ns = max(1, int(N * 0.01))
    state = [(None, None) for _ in range(W)]
    cap, pending, overflows = None, None, 0
    steps = []
    for s in range(STEPS):
        sel = []
        for r in range(W):
            res, acc = state[r]
            t, res, acc = O.dgc_memory_compensate(_grad(r, s), res, acc, MOM)
            sidx = torch.empty([ns]).uniform_(0, N, generator=gens[r]).type(torch.long).numpy()
            vals, idx, _, _ = O.dgc_compress(t, sidx, RATIO)
            sel.append((vals, idx, res, acc))
        counts = [v.size for v, _, _, _ in sel]
        mx = max(counts)
        if exchange == "capacity" and overflow == "defer" and pending is not None:
            pmx, pover = pending
            if pover:
                overflows += 1
            if pover or _grow(pmx, margin) * 4 < cap:
                cap = _grow(pmx, margin)
        if exchange == "counts" or cap is None:
            send = None                                     # everything travels
            if exchange == "capacity":
                cap = _grow(mx, margin)
        elif overflow == "retry":
            send = None
            if mx > cap:
                overflows += 1
                cap = _grow(mx, margin)
            elif _grow(mx, margin) * 4 < cap:
                cap = _grow(mx, margin)
        else:
            send = cap
            pending = (mx, mx > cap)
        decs = []
        for r in range(W):
            vals, idx, res, acc = sel[r]
            if send is not None:
                vals, idx = vals[:send], idx[:send]
            decs.append(O.sparse_decode(vals, idx, N))
            keep = np.ones(N, dtype=bool)
            keep[idx] = False                               # zeroed only where an entry travelled
            state[r] = O.dgc_memory_update(res, acc, ~keep)
        out = (O.python_sum(decs) / F32(W)).astype(F32)
        steps.append((out, [st[0] for st in state], [st[1] for st in state], max(counts), cap))
    return steps, overflows


@pytest.mark.parametrize("mode", [("counts", 1.25, "defer"), ("capacity", 1.0, "retry"),
                                  ("capacity", 1.0, "defer"), ("capacity", 1.5, "defer")])
def test_dgc_world2_exchange_modes(mode):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(os.path.join(tmp, "rdv"), tmp, mode), nprocs=W, join=True)
        got = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(W)]
    steps, overflows = _expected(mode)
    for s, (out, rs, accs, mx, cap) in enumerate(steps):
        for r in range(W):
            assert same_bits(got[r][f"out{s}"], out), (mode, s, r, mx, cap)
            assert same_bits(got[r][f"r{s}"], rs[r]), (mode, s, r)
            assert same_bits(got[r][f"a{s}"], accs[r]), (mode, s, r)
    for r in range(W):
        assert int(got[r]["overflows"][0]) == overflows, (mode, [int(g["overflows"][0]) for g in got], overflows)
    if mode[0] == "counts":
        assert int(got[0]["host_reads"][0]) == STEPS              # one read per step (the W counts)
    elif mode[2] == "defer":
        assert int(got[0]["host_reads"][0]) == 1                  # only the name's first step reads
    if mode == ("capacity", 1.0, "defer") or mode == ("capacity", 1.0, "retry"):
        assert overflows >= 1, "the margin-1.0 run was meant to overflow at least once"
