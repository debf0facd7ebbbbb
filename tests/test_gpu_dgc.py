"""GPU parity of DGC (grace_amd/csrc/dgc.hip, grace_amd/dist/{compressor,memory}/dgc.py) against
the reference's golden vectors and the oracle: with the reference's sample indices injected, the
payload (values, int64 indices, ascending) and the memory states are bit-exact."""
import numpy as np
import pytest
import torch

from grace_amd import ops
from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def test_dgc_compress_golden(golden):
    cases = golden.cases("dgc", codec="dgc")
    assert cases
    for c in cases:
        vals, idx, _ = ops.dgc_compress(_t(c["x"].ravel()), c.meta["ratio"], sample_idx=_t(c["sample_idx"]))
        assert np.array_equal(_np(idx), c["idx"]), c.name
        assert same_bits(_np(vals), c["vals"]), c.name
        dec = _np(ops.sparse_decode(vals, idx, c["x"].size))
        assert same_bits(dec, c["dec"].ravel()), c.name


def test_dgc_memory_sequence_golden(golden):
    from grace_amd.dist.compressor.dgc import DgcCompressor
    from grace_amd.dist.memory.dgc import DgcMemory
    for c in golden.cases("dgc", codec="dgc_memory"):
        comp, mem = DgcCompressor(c.meta["ratio"], rng="torch_cpu"), DgcMemory(c.meta["momentum"], False, 1)
        for s in range(c.meta["steps"]):
            t = mem.compensate(_t(c[f"g{s}"]), "w")
            assert same_bits(_np(t), c[f"t{s}"]), (c.name, s)
            torch.manual_seed(int(c[f"seed{s}"][0]))
            (vals, idx), ctx = comp.compress(t, "w")
            assert np.array_equal(_np(idx), c[f"idx{s}"]) and same_bits(_np(vals), c[f"vals{s}"]), (c.name, s)
            mem.update(t, "w", comp, (vals, idx), ctx)
            assert same_bits(_np(mem.residuals["w"]), c[f"res{s}"]), (c.name, s)
            assert same_bits(_np(mem.gradients["w"]), c[f"grad{s}"]), (c.name, s)


@pytest.mark.parametrize("n,ratio", [((1 << 20) + 3, 0.01), (5_000_000, 0.001), (300_000, 0.3)])
def test_dgc_large_vs_oracle(n, ratio):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    x[rng.integers(0, n, 50)] = np.round(x[rng.integers(0, n, 50)], 1)     # some exact duplicates
    ns = max(1, int(n * 0.01))
    sidx = rng.integers(0, n, ns).astype(np.int64)
    vals, idx, meta = ops.dgc_compress(_t(x), ratio, sample_idx=_t(sidx))
    ev, ei, mask, thr = O.dgc_compress(x, sidx, ratio)
    assert np.array_equal(_np(idx), ei)
    assert same_bits(_np(vals), ev)
    assert _np(meta[4:8].view(torch.float32))[0] == thr
    # the mask update agrees with the oracle's mask
    r = _t(rng.standard_normal(n).astype(np.float32))
    a = _t(x)
    r0 = _np(r)
    ops.dgc_mask_update(a, r, a, meta)
    er, ea = O.dgc_memory_update(r0, x, mask)
    assert same_bits(_np(r), er) and same_bits(_np(a), ea)


def test_dgc_device_rng_and_step():
    """Device sampling: the selection size lands in the reference's [0.7, 1.3] x target band on
    Gaussian data; Allgather(DGC, DgcMemory) steps run through the helper at world 1."""
    from grace_amd.dist.helper import grace_from_params
    n, ratio = 2_000_000, 0.01
    x = _t(np.random.default_rng(7).standard_normal(n).astype(np.float32))
    vals, idx, _ = ops.dgc_compress(x, ratio, seed=123)
    m = vals.numel()
    assert 0.7 * n * ratio <= m <= 1.3 * n * ratio
    assert torch.all(idx[1:] > idx[:-1])
    comm = grace_from_params({"compressor": "dgc", "compress_ratio": ratio, "memory": "dgc",
                              "communicator": "allgather", "world_size": 1})
    for s in range(3):
        g = _t(np.random.default_rng(10 + s).standard_normal(n).astype(np.float32))
        out = comm.step(g, "w")
        assert out.shape == g.shape and torch.isfinite(out).all()
        nz = int((out != 0).sum())
        assert 0 < nz <= 1.3 * n * ratio + 1


def test_dgc_nan_sample_selects_nothing():
    x = np.random.default_rng(3).standard_normal(10000).astype(np.float32)
    x[17] = np.nan
    sidx = np.full(100, 17, dtype=np.int64)
    vals, idx, _ = ops.dgc_compress(_t(x), 0.1, sample_idx=_t(sidx))
    ev, ei, _, _ = O.dgc_compress(x, sidx, 0.1)
    assert vals.numel() == ev.size == 0


@pytest.mark.parametrize("n", [1000, 4097, (1 << 20) + 3])
@pytest.mark.parametrize("rng", ["device", "torch_cpu"])
def test_dgc_world1_fused_step_equals_unfused(n, rng):
    """Allgather(DgcCompressor, DgcMemory).step at world 1 through the one-pass path
    (grace_dgc_select + grace_dgc_step_w1) against the reference's four calls on the same engine:
    outputs and both memory states bit-exact over 3 steps (momentum state carried)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.dgc import DgcCompressor
    from grace_amd.dist.memory.dgc import DgcMemory
    gs = [np.random.default_rng(n + s).standard_normal(n).astype(np.float32) for s in range(3)]
    runs = []
    for fused in (True, False):
        torch.manual_seed(5)
        comm = Allgather(DgcCompressor(0.01, rng=rng), DgcMemory(0.9, False, 1), 1)
        outs = []
        for s in range(3):
            g = _t(gs[s])
            if fused:
                out = comm.step(g, "w")
            else:
                t = comm.memory.compensate(g, "w")
                payload, ctx = comm.compressor.compress(t, "w")
                comm.memory.update(t, "w", comm.compressor, payload, ctx)
                out = comm.send_receive(payload, "w", ctx)
            outs.append(_np(out))
        runs.append((outs, _np(comm.memory.residuals["w"]), _np(comm.memory.gradients["w"])))
    (fo, fr, fa), (uo, ur, ua) = runs
    for s in range(3):
        assert same_bits(fo[s], uo[s]), s
    assert same_bits(fr, ur) and same_bits(fa, ua)
    assert np.count_nonzero(fo[-1]) > 0


def _unfused_w1(g, r, a, has, m, ratio, sidx):
    """compensate (in place, on copies) + select + step_w1: the multi-pass world-1 step."""
    r, a = (r.clone(), a.clone()) if has else (torch.empty_like(g), torch.empty_like(g))
    ops.dgc_compensate(g, r, a, has, m)
    ws = ops.dgc_select(a, ratio, sample_idx=sidx)
    out = ops.dgc_step_w1(a, r, a, ws)
    return out, r, a


@pytest.mark.parametrize("case", ["normal", "sample_top", "sample_nan", "specials", "unaligned"])
def test_dgc_w1_speculative_pass_equals_multipass(case):
    """grace_dgc_step_w1_fused selects at the sampled threshold in one pass and redoes the step
    through the gated full adjustment loop when that threshold does not stand: a sample of the
    largest element (count far below 0.7 k: the loop runs), a NaN sample, inf / NaN / -0 in the
    gradient, an unaligned length; three steps with the momentum state carried, out and both
    memory states bit-identical to the multi-pass step."""
    n = (1 << 20) + (3 if case == "unaligned" else 0)
    ratio, m = 0.01, 0.9
    rng = np.random.default_rng(len(case))
    r = a = None
    for s in range(3):
        g0 = rng.standard_normal(n).astype(np.float32)
        if case == "specials":
            g0[rng.choice(n, 5, replace=False)] = np.inf
            g0[rng.choice(n, 5, replace=False)] = -np.inf
            g0[rng.choice(n, 3, replace=False)] = np.nan
            g0[rng.choice(n, 50, replace=False)] = -0.0
        g = _t(g0)
        ns = max(1, int(n * 0.01))
        sidx = rng.integers(0, n, ns).astype(np.int64)
        if case == "sample_top":
            sidx[:] = int(np.argmax(np.abs(g0)))
        if case == "sample_nan":
            g0[7] = np.nan
            g = _t(g0)
            sidx[:] = 7
        has = s > 0
        eo, er, ea = _unfused_w1(g, r, a, has, m, ratio, _t(sidx))
        out, r_new, a_new = ops.dgc_step_w1_fused(g, r, a, has, m, ratio, sample_idx=_t(sidx))
        assert same_bits(_np(out), _np(eo)), (case, s)
        assert same_bits(_np(r_new), _np(er)) and same_bits(_np(a_new), _np(ea)), (case, s)
        r, a = r_new, a_new


@pytest.mark.parametrize("case", ["normal", "ties", "zeros", "inf", "nan", "tiny", "ks1", "ksall", "denorm"])
def test_dgc_sample_kth_equals_topk_min(case):
    """grace_dgc_sample_kth = torch.topk(sample, ks)[0].min() (dgc.py:20-21), bit for bit, NaN
    included: the radix select every DGC path takes its sampled threshold from."""
    gen = torch.Generator().manual_seed(11)
    ns, ks = 671088, 6710
    x = torch.randn(ns, generator=gen).abs()
    if case == "ties":
        x = torch.randint(0, 7, (ns,), generator=gen).float()
    elif case == "zeros":
        x = torch.zeros(ns)
    elif case == "inf":
        x[torch.randint(0, ns, (9000,), generator=gen)] = float("inf")
    elif case == "nan":
        x[12345] = float("nan")
    elif case == "tiny":
        ns, ks = 3, 2
        x = torch.tensor([0.5, 2.0, 1.0])
    elif case == "ks1":
        ks = 1
    elif case == "ksall":
        ns = 5000
        x, ks = x[:ns], 5000
    elif case == "denorm":
        x = (torch.rand(ns, generator=gen) * 1e-39).abs()
    xd = _t(x.numpy())
    for _ in range(2):   # the state is left zeroed: a second call gives the same answer
        got = _np(ops.dgc_sample_kth(xd, ks))
        want = torch.topk(x, ks)[0].min().reshape(1).numpy()
        if np.isnan(want[0]):
            assert np.isnan(got[0])
        else:
            assert same_bits(got, want), (case, got, want)


def test_dgc_thresholds_same_with_either_sample_select():
    """The three-digit select and the top-k engine's values give DGC the same threshold and payload
    (ops.DGC_SAMPLE_KTH switched in one process)."""
    gen = torch.Generator().manual_seed(5)
    t = _t((torch.randn(1 << 22, generator=gen) * 0.01).numpy())
    res = []
    for kth in (True, False):
        ops.DGC_SAMPLE_KTH = kth
        try:
            vals, idx, meta = ops.dgc_compress(t, 0.01, seed=3)
        finally:
            ops.DGC_SAMPLE_KTH = True
        res.append((_np(vals), _np(idx), _np(meta.view(torch.int32))))
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
