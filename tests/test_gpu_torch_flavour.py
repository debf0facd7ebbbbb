"""GPU parity of the Horovod-flavour codecs (grace_amd/torch/compressor/*) against golden vectors
captured from the reference's grace_dl/torch modules (tests/golden/gen_golden.py, store
``torchflav``).  Those reference modules import no horovod, so they ran here on CPU.

Bars: codewords / indices / values / decoded tensors bit-exact (with the reference's uniforms or
seed injected); the device-computed global QSGD norm (f64 accumulation) within 1 ulp of the exact
norm and rel 4e-6 of torch's f32 ``tensor.norm()`` (whose own error grows with n).
PowerSGD's torch flavour needs horovod: parity unpinned, checked against the oracle restatement
within the f32 bar rel 1e-5 * sqrt(m).
"""
import numpy as np
import pytest
import torch

from grace_amd import ops
from oracle import grace_oracle as O
from tests.golden_util import same_bits, topk_sets_match

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def test_qsgd_global_norm_golden(golden):
    from grace_amd.torch.compressor.qsgd import QSGDCompressor
    cases = golden.cases("torchflav", codec="qsgd")
    assert cases
    for c in cases:
        q = c.meta["quantum_num"]
        x = c["x"].ravel()
        u = _t(c["u"])
        # the reference's norm injected: codewords bit-exact
        codes, norm = ops.qsgd_global_compress(_t(x), q, u=u, norm_in=_t(c["norm"]))
        assert same_bits(_np(codes), c["codes"].ravel()), c.name
        assert same_bits(_np(norm), c["norm"].ravel()), c.name
        # the device norm (f64 accumulation): within 1 ulp of the exactly rounded norm, and within
        # rel 4e-6 of torch's f32 CPU reduction, whose own rounding error grows with n (13 ulp at
        # n = 100003); codewords bit-exact given the device norm
        codes2, norm2 = ops.qsgd_global_compress(_t(x), q, u=u)
        exact = np.float32(np.sqrt(np.sum(x.astype(np.float64) ** 2)))
        assert ops.isclose_f32_ulps(_np(norm2), np.array([exact]), 1), (c.name, _np(norm2), exact)
        assert np.allclose(_np(norm2), c["norm"].ravel(), rtol=4e-6, atol=0), (c.name, _np(norm2), c["norm"])
        exp, _ = O.qsgd_global_compress(x, c["u"], q, norm=_np(norm2))
        assert same_bits(_np(codes2), exp), c.name
        # decompress of the reference payload: bit-exact, through the compressor class
        comp = QSGDCompressor(q)
        dec = comp.decompress((_t(c["codes"].ravel()), _t(c["norm"])), torch.Size(c["x"].shape))
        assert same_bits(_np(dec), c["dec"]), c.name
        # the class in torch-CPU-generator mode consumes the same uniforms as the reference
        comp = QSGDCompressor(q, rng="torch_cpu")
        torch.manual_seed(c.meta["seed"])
        (codes3, norm3), shape = comp.compress(_t(c["x"]), "w")
        assert shape == torch.Size(c["x"].shape)
        exp3, _ = O.qsgd_global_compress(x, c["u"], q, norm=_np(norm3))
        assert same_bits(_np(codes3), exp3), c.name


def test_threshold_strict_golden(golden):
    from grace_amd.torch.compressor.threshold import ThresholdCompressor
    cases = golden.cases("torchflav", codec="threshold")
    assert cases
    for c in cases:
        comp = ThresholdCompressor(c.meta["threshold"])
        (vals, idx), ctx = comp.compress(_t(c["x"]), "w")
        assert idx.dtype == torch.int64
        assert ctx == (torch.Size(c["x"].shape), c["x"].size)
        assert np.array_equal(_np(idx), c["idx"]), c.name
        assert same_bits(_np(vals), c["vals"]), c.name
        assert same_bits(_np(comp.decompress([vals, idx], ctx)), c["dec"]), c.name


def test_randomk_randperm_golden(golden):
    from grace_amd.torch.compressor.randomk import RandomKCompressor
    cases = golden.cases("torchflav", codec="randomk")
    assert cases
    comps = {}
    for c in cases:   # generation order: one compressor per ratio, its global_step shared across names
        comp = comps.setdefault(c.meta["ratio"], RandomKCompressor(c.meta["ratio"], rng="torch_cpu"))
        assert sum(bytes(c.meta["name"], "utf8"), comp.global_step) == c.meta["seed"]
        (vals,), ctx = comp.compress(_t(c["x"]), c.meta["name"])
        idx, numel, shape = ctx
        assert np.array_equal(_np(idx), c["idx"]), c.name
        assert same_bits(_np(vals), c["vals"]), c.name
        assert same_bits(_np(comp.decompress([vals], ctx)), c["dec"]), c.name


@pytest.mark.parametrize("numel,ratio", [(1, 0.3), (129, 0.3), (4099, 1.0), (100003, 0.01), (1 << 22, 0.3)])
def test_randomk_device_permutation_properties(numel, ratio):
    """Device mode: k DISTINCT indices in [0, numel) (no replacement), identical for the same seed
    (every rank derives the same set), different seeds give different sets, values gathered."""
    from grace_amd.torch.compressor.randomk import RandomKCompressor
    k = O.ratio_k(numel, ratio)
    a = _np(ops.randomk_perm_indices(1234, numel, k, DEV))
    b = _np(ops.randomk_perm_indices(1234, numel, k, DEV))
    assert a.size == k and np.array_equal(a, b)
    assert a.min() >= 0 and a.max() < numel
    assert np.unique(a).size == k
    if k < numel:
        assert not np.array_equal(a, _np(ops.randomk_perm_indices(1235, numel, k, DEV)))
    if ratio == 1.0:
        assert np.array_equal(np.sort(a), np.arange(numel))
    x = np.random.default_rng(numel).standard_normal(numel).astype(np.float32)
    comp = RandomKCompressor(ratio)
    (vals,), (idx, n, shape) = comp.compress(_t(x), "w")
    assert same_bits(_np(vals), x[_np(idx)])
    dec = _np(comp.decompress([vals], (idx, n, shape)))
    exp = np.zeros(numel, np.float32)
    exp[_np(idx)] = x[_np(idx)]
    assert same_bits(dec, exp)


def test_topk_int64_golden(golden):
    from grace_amd.torch.compressor.topk import TopKCompressor
    cases = golden.cases("torchflav", codec="topk")
    assert cases
    for c in cases:
        comp = TopKCompressor(c.meta["ratio"])
        x = c["x"]
        (vals, idx), ctx = comp.compress(_t(x), "w")
        assert idx.dtype == torch.int64 and ctx == (x.size, torch.Size(x.shape))
        k = O.ratio_k(x.size, c.meta["ratio"])
        assert topk_sets_match(x.ravel(), _np(idx), c["idx"], k), c.name
        assert same_bits(_np(vals), x.ravel()[_np(idx)]), c.name
        dec = _np(comp.decompress([vals, idx], ctx))
        exp = O.sparse_decode(_np(vals), _np(idx), x.size).reshape(x.shape)
        assert same_bits(dec, exp), c.name
        if np.array_equal(np.sort(_np(idx)), np.sort(c["idx"])):
            assert same_bits(dec, c["dec"]), c.name


def test_terngrad_torch_flavour_golden(golden):
    from grace_amd.torch.compressor.terngrad import TernGradCompressor
    cases = golden.cases("torchflav", codec="terngrad")
    assert cases
    for c in cases:
        x = c["x"].ravel()
        clip = np.array([O.terngrad_clip(x)], dtype=np.float32)
        codes, scal = ops.terngrad_compress(_t(x), clip=_t(clip), u=_t(c["u"]))
        assert np.array_equal(_np(codes), c["codes"].ravel()), c.name
        assert same_bits(_np(scal), c["scalar"].ravel()), c.name
        dec = TernGradCompressor().decompress((_t(c["codes"].ravel()), _t(c["scalar"].ravel())),
                                              torch.Size(c["x"].shape))
        assert same_bits(_np(dec), c["dec"]), c.name


def test_onebit_torch_flavour_fixed_decode(golden):
    from grace_amd.torch.compressor.onebit import OneBitCompressor
    for c in golden.cases("sign", codec="onebit"):
        comp = OneBitCompressor()
        (mask0, m0, m1), shape = comp.compress(_t(c["x"]), "w")
        assert np.array_equal(_np(mask0), c["mask0"]), c.name
        assert ops.isclose_f32_ulps(_np(m0), c["mean0"], 4) and ops.isclose_f32_ulps(_np(m1), c["mean1"], 4), c.name
        dec = comp.decompress((mask0, _t(c["mean0"]), _t(c["mean1"])), shape)   # the reference's means
        assert same_bits(_np(dec), c["dec_fixed"]), c.name


@pytest.mark.parametrize("shape,rank", [((64, 48), 2), ((256, 256), 4), ((16, 3, 3, 3), 1)])
def test_powersgd_torch_flavour_vs_oracle(shape, rank):
    """q comes from the memory and is orthogonalised IN PLACE, P and Q are averaged (W = 1 here),
    q_memory[name] becomes Q; rank = the memory's compress_rank.  Parity unpinned (horovod)."""
    from grace_amd.torch.compressor.powersgd import PowerSGDCompressor
    from grace_amd.torch.memory.powersgd import PowerSGDMemory
    rng = np.random.default_rng(rank)
    x = rng.standard_normal(shape).astype(np.float32)
    comp = PowerSGDCompressor()
    mem = PowerSGDMemory(comp.q_memory, compress_rank=rank)
    t = mem.compensate(_t(x), "w")                       # draws q into the shared q_memory
    n, m = shape[0], int(np.prod(shape[1:]))
    assert tuple(comp.q_memory["w"].shape) == (m, min(n, m, rank))
    q0 = _np(comp.q_memory["w"]).copy()
    payload, ctx = comp.compress(t, "w")
    p, q, shp = ctx
    p_or, q_or = O.powersgd_compress(x.reshape(n, m), O.orthogonalize(q0))
    tol = 1e-5 * np.sqrt(m)
    assert np.allclose(_np(p), p_or, rtol=tol, atol=tol * np.abs(p_or).max())
    assert np.allclose(_np(q), q_or, rtol=tol, atol=tol * np.abs(q_or).max())
    assert comp.q_memory["w"] is q
    dec = _np(comp.decompress(payload, ctx))
    exp = O.powersgd_decode(p_or, q_or).reshape(shape)
    assert np.allclose(dec, exp, rtol=tol, atol=tol * np.abs(exp).max())
    mem.update(t, "w", comp, payload, ctx)
    assert np.allclose(_np(mem.residuals["w"]), x - exp, rtol=tol, atol=tol * np.abs(x).max())


def test_helper_builds_torch_flavour_codecs():
    from grace_amd.torch.helper import grace_from_params
    from grace_amd.torch.compressor.qsgd import QSGDCompressor
    from grace_amd.torch.compressor.threshold import ThresholdCompressor
    g = grace_from_params({"compressor": "qsgd", "memory": "none", "communicator": "allgather"})
    assert type(g.compressor) is QSGDCompressor
    g = grace_from_params({"compressor": "threshold", "memory": "residual", "communicator": "allreduce"})
    assert type(g.compressor) is ThresholdCompressor
    x = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    handles, ctx = g.send_step(_t(x), "w")
    out = _np(g.receive_step(handles, ctx))
    v, i = O.threshold_select_strict(x, 0.01)
    assert same_bits(out, O.sparse_decode(v, i, x.size))
