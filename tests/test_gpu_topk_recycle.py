"""Recycled dense output of the world-1 top-k step (ops.OutputRecycler, grace_topk_residual_step_carry
with prev_idx): when the caller drops a step's result without modifying it, the next step of the
same name gets that tensor back, the bracket launch zeroes the previous payload positions and the
main pass writes only its own selection.  Every result must equal the dense-write path and the
oracle bit for bit, whatever the caller does with its results: keep them, keep a view, edit them
in place, or take the exact fallback (a bucket of ties) in between."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _np(t):
    return t.detach().cpu().numpy()


def _comm(recycle):
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    return Allgather(TopKCompressor(0.01, recycle_output="always" if recycle else False), ResidualMemory(), 1)


def _grads(n, steps, seed, ties_at=()):
    rng = np.random.default_rng(seed)
    out = []
    for s in range(steps):
        g = rng.standard_normal(n).astype(np.float32)
        if s in ties_at:                      # 99.9 % exact zeros: the k-th key is 0, exact fallback
            g[rng.random(n) < 0.999] = 0.0
        out.append(g)
    return out


@pytest.mark.parametrize("n", [(1 << 20) + 7, 1 << 22])
def test_recycled_output_equals_dense_and_oracle(n):
    gs = _grads(n, 6, 3, ties_at=(3,))
    rec, ref = _comm(True), _comm(False)
    r_or = None
    recycled = 0
    for s, g in enumerate(gs):
        gt = torch.from_numpy(g).to(DEV)
        before = rec.compressor._recycler._hit.get("b")
        o1 = rec.step(gt, "b")
        if before is not None and o1.data_ptr() == before[0].data_ptr():
            recycled += 1
        o2 = ref.step(gt, "b")
        _, _, _, r_or, out_or = O.topk_residual_step(g, r_or, 0.01)
        a = _np(o1)
        assert same_bits(a, _np(o2)), s
        assert same_bits(a, out_or), s
        assert same_bits(_np(rec.memory.residuals["b"]), r_or), s
        del o1, o2                            # dropped: the next step may recycle it
    assert recycled == len(gs) - 1            # every step after the first reused its buffer


def test_recycling_never_touches_a_result_the_caller_holds_or_edited():
    n = (1 << 20) + 3
    gs = _grads(n, 6, 4)
    rec = _comm(True)
    r_or = None
    kept = {}
    ptr = {}
    for s, g in enumerate(gs):
        o = rec.step(torch.from_numpy(g).to(DEV), "b")
        ptr[s] = o.data_ptr()
        _, _, _, r_or, out_or = O.topk_residual_step(g, r_or, 0.01)
        assert same_bits(_np(o), out_or), s
        if s == 0:
            kept[s] = (o, out_or)                    # held: never recycled
        elif s == 1:
            kept[s] = (o.view(-1)[5:], out_or[5:])   # only a view held
        elif s == 2:
            o.mul_(2.0)                              # edited in place, then dropped
        del o
    for s, (t, exp) in kept.items():
        assert same_bits(_np(t), exp), f"held result of step {s} was overwritten"
    assert ptr[1] != ptr[0] and ptr[2] != ptr[1]      # held results were not handed back
    assert ptr[3] != ptr[2]                           # the edited one was not either
    assert ptr[4] == ptr[3] and ptr[5] == ptr[4]      # dropped, unmodified ones are


def test_recycled_output_two_names_and_streams():
    """Buckets on two streams keep separate recycled outputs; results stay exact."""
    n = (1 << 20) + 11
    gs = [_grads(n, 4, 10 + j) for j in range(2)]
    rec = _comm(True)
    streams = [torch.cuda.Stream() for _ in range(2)]
    r_or = [None, None]
    for s in range(4):
        outs = []
        for j in range(2):
            with torch.cuda.stream(streams[j]):
                outs.append(rec.step(torch.from_numpy(gs[j][s]).to(DEV), f"b{j}"))
        torch.cuda.synchronize()
        for j in range(2):
            _, _, _, r_or[j], out_or = O.topk_residual_step(gs[j][s], r_or[j], 0.01)
            assert same_bits(_np(outs[j]), out_or), (s, j)
        del outs


def test_randomk_recycled_output_equals_dense():
    """World-1 Allgather(RandomK 1 %, Residual).step with the recycled output (the previous grouping
    of the drawn indices clears the old non-zeros; duplicates and re-drawn positions included)
    equals the dense-write step bit for bit, and held results are never touched."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n = (1 << 20) + 5
    rec = Allgather(RandomKCompressor(0.01, recycle_output=True), ResidualMemory(), 1)
    ref = Allgather(RandomKCompressor(0.01, recycle_output=False), ResidualMemory(), 1)
    gs = _grads(n, 7, 21)
    held = []
    hits = 0
    for s, g in enumerate(gs):
        gt = torch.from_numpy(g).to(DEV)
        o1 = rec.step(gt, "b")
        o2 = ref.step(gt, "b")
        assert same_bits(_np(o1), _np(o2)), s
        assert same_bits(_np(rec.memory.residuals["b"]), _np(ref.memory.residuals["b"])), s
        if s == 2:
            held.append((o1, _np(o2).copy()))
        del o1, o2
    hits = rec.compressor._recycler.hits
    assert hits >= 4
    for t, exp in held:
        assert same_bits(_np(t), exp)


def test_topk_nomem_recycled_output_equals_dense():
    """The no-memory world-1 step (the default recycling path) against the dense-write step and the
    oracle's compress + decompress over steps with dropped results, a held one and an exact-fallback
    bucket (99.9 % zeros) in between."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = (1 << 20) + 9
    rec = Allgather(TopKCompressor(0.01), NoneMemory(), 1)
    ref = Allgather(TopKCompressor(0.01, recycle_output=False), NoneMemory(), 1)
    gs = _grads(n, 7, 33, ties_at=(4,))
    held = None
    for s, g in enumerate(gs):
        gt = torch.from_numpy(g).to(DEV)
        o1 = rec.step(gt, "b")
        o2 = ref.step(gt, "b")
        _, v_or, i_or, _, out_or = O.topk_residual_step(g, None, 0.01)
        assert same_bits(_np(o1), _np(o2)), s
        assert same_bits(_np(o1), out_or), s
        if s == 2:
            held = (o1, out_or)
        del o1, o2
    assert rec.compressor._recycler.hits >= 4
    assert same_bits(_np(held[0]), held[1])
