"""GPU parity of PowerSGD (grace_amd/csrc/powersgd.hip, f32 MFMA) against golden vectors, within
the f32 tolerance rel <= 1e-5 * sqrt(m) stated in SURVEY.md §8a (different summation orders)."""
import numpy as np
import pytest
import torch

from grace_amd import ops
from oracle import grace_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def _close(a, b, m, scale=None):
    tol = 1e-5 * np.sqrt(m)
    scale = np.abs(b).max() if scale is None else scale
    return np.allclose(a, b, rtol=tol, atol=tol * max(scale, 1e-30))


@pytest.mark.parametrize("shape", [(64, 48), (33, 17), (256, 256), (100, 1000), (4096, 4096)])
@pytest.mark.parametrize("r", [1, 2, 4])
def test_p_and_qt_vs_numpy(shape, r):
    rng = np.random.default_rng(shape[0] + r)
    M = rng.standard_normal(shape).astype(np.float32)
    q = rng.standard_normal((shape[1], r)).astype(np.float32)
    P = _np(ops.powersgd_p(_t(M), _t(q)))
    Pe = (M.astype(np.float64) @ q.astype(np.float64))
    assert _close(P, Pe, shape[1])
    Q = _np(ops.powersgd_qt(_t(M), _t(P)))
    Qe = M.T.astype(np.float64) @ P.astype(np.float64)
    assert _close(Q, Qe, shape[0])
    out, res = ops.powersgd_outer(_t(P), _t(Q), _t(M), want_out=True, want_residual=True)
    Oe = P.astype(np.float64) @ Q.T.astype(np.float64)
    assert _close(_np(out), Oe, r)
    assert _close(_np(res), M - _np(out), 1, scale=np.abs(M).max())


def test_orthogonalize_golden(golden):
    for c in golden.cases("powersgd", codec="orthogonalize"):
        a = _t(c["a"])
        ops.orthogonalize_(a)
        assert np.allclose(_np(a), c["out"], rtol=1e-4, atol=1e-5), c.name


def test_powersgd_compressor_golden(golden):
    from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
    for c in golden.cases("powersgd", codec="powersgd"):
        if "steps" in c.meta:
            continue
        comp = PowerSGDCompressor(rank=c.meta["rank"], use_memory=True, world_size=1)
        comp.q_memory["w"] = _t(c["q0"])
        payload, ctx = comp.compress(_t(c["x"]), "w")
        p, q, shape = ctx
        m = int(np.prod(c["x"].shape[1:]))
        assert _close(_np(p), c["p"], m), c.name
        assert _close(_np(q), c["q"], m), c.name
        dec = _np(comp.decompress(payload, ctx))
        assert dec.shape == c["dec"].shape
        assert _close(dec, c["dec"], m), c.name


def test_powersgd_memory_allreduce_sequence(golden):
    """Two Allreduce(PowerSGD, PowerSGDMemory) steps with the reference's q draws injected."""
    from grace_amd.dist.communicator.allreduce import Allreduce
    from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
    from grace_amd.dist.memory.powersgd import PowerSGDMemory
    c = golden.case("powersgd", "powersgd_memory_seq")
    comp = PowerSGDCompressor(rank=2, use_memory=True, world_size=1)
    mem = PowerSGDMemory(comp.q_memory, compress_rank=2)
    comm = Allreduce(comp, mem, 1)
    for s in range(2):
        g = _t(c[f"g{s}"])
        t = mem.compensate(g, "w")
        q0 = _t(c[f"qdraw{s}"])
        ops.orthogonalize_(q0)
        comp.q_memory["w"] = q0      # the reference drew and orthogonalised this q in compress
        payload, ctx = comp.compress(t, "w")
        mem.update(t, "w", comp, payload, ctx)
        out = comm.send_receive(payload, "w", ctx)
        assert np.allclose(_np(t), c[f"t{s}"], rtol=1e-5, atol=1e-5)
        assert np.allclose(_np(ctx[0]), c[f"p{s}"], rtol=1e-3, atol=1e-4)
        assert np.allclose(_np(mem.residuals["w"]), c[f"res{s}"], rtol=1e-3, atol=1e-3)
        assert np.allclose(_np(out), c[f"dec{s}"], rtol=1e-3, atol=1e-3)


def test_one_dim_passthrough():
    from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
    comp = PowerSGDCompressor(rank=4)
    x = _t(np.arange(10, dtype=np.float32))
    payload, ctx = comp.compress(x, "b")
    assert ctx is None and comp.decompress(payload, ctx) is x


@pytest.mark.parametrize("n,r", [(4096, 4), (5000, 3), (100, 1), (9000, 8), (300, 16)])
def test_orthogonalize_shapes_and_fused_draw(n, r):
    """Register-resident (n <= 4096) and chunked (taller) orthogonalisation against a float64
    MGS, and the fused draw == draw then orthogonalise."""
    rng = np.random.default_rng(n + r)
    a = rng.standard_normal((n, r)).astype(np.float32)
    out = _np(ops.orthogonalize_(_t(a)))
    exp = a.astype(np.float64)
    for i in range(r):
        exp[:, i] /= np.sqrt(np.sum(exp[:, i] ** 2))
        if i + 1 < r:
            exp[:, i + 1:] -= np.sum(exp[:, i:i + 1] * exp[:, i + 1:], axis=0) * exp[:, i:i + 1]
    assert np.allclose(out, exp, rtol=1e-4, atol=1e-5)
    fused = _np(ops.normal_orthogonal((n, r), 77, "cuda"))
    ref = _np(ops.orthogonalize_(ops.normal((n, r), 77, "cuda")))
    assert np.allclose(fused, ref, rtol=1e-5, atol=1e-6)
    assert np.allclose(fused.T.astype(np.float64) @ fused, np.eye(r), atol=1e-4)
