"""Buffer-pair placement of the world-1 fused top-k step (ops.pick_pair, DESIGN §4 "Buffer-pair
placement"): a large bucket's first step probes residual / output allocation pairs and keeps the
fastest; later steps rewrite the kept output in full.  Results must stay bit-exact against the
oracle's Allgather(TopK, ResidualMemory).step sequence (grace_dl/dist/compressor/topk.py:32-42,
memory/residual.py:10-20), a result the caller holds must never be reused, and the probe must leave
nothing of its own in the step's buffers."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu


def _g(n, s):
    return np.random.default_rng(900 + s).standard_normal(n).astype(np.float32)


@pytest.mark.parametrize("hold", [False, True])
def test_pair_placement_steps_exact(hold):
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    assert ops.PLACE_PROBE
    n, ratio = ops.PLACE_MIN_N + 4096, 0.01
    comm = Allgather(TopKCompressor(ratio), ResidualMemory(), 1)
    r_or = None
    held = []
    for s in range(4):
        g = _g(n, s)
        out = comm.step(torch.from_numpy(g).cuda(), "bucket")
        _, _, _, r_or, out_or = O.topk_residual_step(g, r_or, ratio)
        o = out.cpu().numpy()
        assert same_bits(o, out_or), s
        assert same_bits(comm.memory.residuals["bucket"].cpu().numpy(), r_or), s
        if hold:
            held.append((out, o.copy()))   # the caller keeps every result: none may be reused
        del out
    probes = comm.compressor.place_probes["bucket"]
    assert len(probes) == ops.PLACE_RES * ops.PLACE_OUT and min(probes) > 0
    rec = comm.compressor._recycler
    if hold:
        assert rec.dense_hits == 0
        for t, o in held:
            assert same_bits(t.cpu().numpy(), o)
    else:
        assert rec.dense_hits == 3 and rec.hits == 0   # steps 2-4 got the kept buffer back, dense


def test_pick_pair_returns_distinct_buffers():
    from grace_amd import ops
    g = torch.randn(ops.PLACE_MIN_N, device="cuda")
    g0 = g.clone()
    r, out, us = ops.pick_pair(g, (0.0, 1.0), (3.0, 8.0))
    torch.cuda.synchronize()
    assert r.data_ptr() != out.data_ptr() and r.numel() == out.numel() == g.numel()
    assert len(us) == 4
    assert torch.equal(g, g0)   # the probe only reads g


def test_pick_pair_without_room_takes_plain_buffers(monkeypatch):
    """A device without room for the trial (here: a spacer larger than the device) gets two plain
    allocations and no probe; the step stays exact."""
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    monkeypatch.setattr(ops, "PLACE_OUT_GIB", (float(1 << 20),))   # an output candidate 1 PiB away
    n, ratio = ops.PLACE_MIN_N, 0.01
    g = torch.randn(n, device="cuda")
    r, out, us = ops.pick_pair(g)
    assert us == [] and r.numel() == out.numel() == n
    comm = Allgather(TopKCompressor(ratio), ResidualMemory(), 1)
    gn = _g(n, 7)
    out = comm.step(torch.from_numpy(gn).cuda(), "b")
    _, _, _, r_or, out_or = O.topk_residual_step(gn, None, ratio)
    assert same_bits(out.cpu().numpy(), out_or)
    assert same_bits(comm.memory.residuals["b"].cpu().numpy(), r_or)
    assert "b" not in comm.compressor.place_probes
