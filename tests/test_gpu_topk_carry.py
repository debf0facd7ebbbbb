"""Residual-sample carry of the fused top-k step (grace_topk_residual_step_carry): the
bracket records t at its sample positions and the finalize the step's selection threshold; the next step's bracket derives r' there from them instead of reading r.  A valid carry
gives the bracket exactly the sample the plain path reads; the carry only steers the sampled
bracket, so every result stays bit-exact against the oracle whatever the carry holds (stale or
garbage carries fall back to the exact path)."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
DEV = "cuda"
SAMPLE_MAX = 131072


def _np(t):
    return t.detach().cpu().numpy()


def sample_positions(n):
    """The bracket's stratified sample positions (topk.hip sample_pos), restated in numpy."""
    sn = min(n, SAMPLE_MAX // 2 if n <= (1 << 24) else SAMPLE_MAX)   # topk.hip bracket_sample_n
    st = n // sn
    s = np.arange(sn, dtype=np.uint64)
    x = ((s * np.uint64(0x9E3779B9) + np.uint64(0x5EED)) & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    m32 = np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16); x = (x * np.uint64(0x7FEB352D)) & m32
    x ^= x >> np.uint64(15); x = (x * np.uint64(0x846CA68B)) & m32
    x ^= x >> np.uint64(16)
    off = (x * np.uint64(st)) >> np.uint64(32)
    return (s * np.uint64(st) + off).astype(np.int64)


def _carried_residual(tp, pos, T):
    key = tp.view(np.uint32).astype(np.uint64) & np.uint64(0x7FFFFFFF)
    comp = (key << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - pos.astype(np.uint64))
    return np.where(comp >= np.uint64(T), tp - tp, tp).astype(np.float32)


def _check_step(g0, r0, k, vals, idx, res, out):
    t = (r0 + g0) if r0 is not None else g0   # beta = gamma = 1: t = 1 * r + 1 * g exactly
    ov, oi = O.topk_select(t, k)
    v, i = _np(vals), _np(idx).astype(np.int64)
    o = np.argsort(i, kind="stable")
    assert np.array_equal(i[o], oi.astype(np.int64)), "index set differs from oracle"
    assert same_bits(v[o], ov), "payload values differ from oracle"
    sel = np.zeros(t.size, dtype=bool)
    sel[oi] = True
    exp_r = t.copy()
    exp_r[sel] = t[sel] - t[sel]
    assert same_bits(_np(res), exp_r), "residual differs"
    if out is not None:
        exp_o = np.zeros_like(t)
        exp_o[sel] = np.float32(0.0) + t[sel]
        assert same_bits(_np(out), exp_o), "dense output differs"
    return exp_r, t


@pytest.mark.parametrize("n", [1 << 25, (1 << 25) + 12345, 1 << 26])
@pytest.mark.parametrize("with_out", [True, False])
def test_carry_records_samples_and_next_step_exact(n, with_out):
    from grace_amd import ops
    k = O.ratio_k(n, 0.01)
    cs = ops.topk_carry_size(n, k)
    assert cs == SAMPLE_MAX + 2
    pos = sample_positions(n)
    assert pos.max() < n and np.all(np.diff(pos) > 0)
    rng = np.random.default_rng(n + with_out)
    carry = torch.full((cs,), float("nan"), device=DEV)
    res = torch.empty(n, device=DEV)
    r_host = None
    for step in range(3):
        g0 = rng.standard_normal(n, dtype=np.float32)
        g = torch.from_numpy(g0).to(DEV)
        out = torch.empty_like(g) if with_out else None
        _, vals, idx = ops.topk_residual_step(g, res, step > 0, 1.0, 1.0, k, out=out, carry=carry,
                                              carry_valid=step > 0)
        torch.cuda.synchronize()
        assert ops.topk_status(n, k, g.device) == 0, "a valid carry must keep the sampled fast path"
        r_host, t = _check_step(g0, r_host, k, vals, idx, res, out)
        # the carry holds t at every sample position and the step's composite threshold: r' at the
        # sample positions follows from them bit for bit
        c = _np(carry)
        assert same_bits(c[:SAMPLE_MAX], t[pos])
        T = int(c[SAMPLE_MAX:].view(np.uint64)[0])
        assert same_bits(r_host[pos], _carried_residual(c[:SAMPLE_MAX], pos, T))
        key = t.view(np.uint32).astype(np.uint64) & np.uint64(0x7FFFFFFF)
        comp = (key << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.arange(n, dtype=np.uint64))
        assert np.count_nonzero(comp >= np.uint64(T)) == k


@pytest.mark.parametrize("fill", [0.0, 1e30, float("nan")])
def test_garbage_carry_still_exact(fill):
    """A carry that does not belong to the residual (all zeros, huge, NaN) misplaces the bracket:
    the step must still be exact (the bracket's exact fallback)."""
    from grace_amd import ops
    n = 1 << 25
    k = O.ratio_k(n, 0.01)
    rng = np.random.default_rng(5)
    g0 = rng.standard_normal(n, dtype=np.float32)
    r0 = (0.5 * rng.standard_normal(n)).astype(np.float32)
    g, res = torch.from_numpy(g0).to(DEV), torch.from_numpy(r0).to(DEV)
    carry = torch.full((ops.topk_carry_size(n, k),), fill, device=DEV)
    out = torch.empty_like(g)
    _, vals, idx = ops.topk_residual_step(g, res, True, 1.0, 1.0, k, out=out, carry=carry, carry_valid=True)
    torch.cuda.synchronize()
    _check_step(g0, r0, k, vals, idx, res, out)


def test_fused_step_carry_tracks_residual_identity_and_version():
    """Communicator.step keeps the carry with the residual; an in-place change of the residual
    (version counter) or a replaced residual invalidates it, and every step stays exact."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n = (1 << 25) + 4
    ratio = 0.01
    k = O.ratio_k(n, ratio)
    mem = ResidualMemory()
    comm = Allgather(TopKCompressor(ratio), mem, 1)
    rng = np.random.default_rng(9)
    r_host = None
    for step in range(5):
        g0 = rng.standard_normal(n, dtype=np.float32)
        res = mem.residuals.get("b")
        if step == 2:
            res.mul_(2.0)          # in place: the carry no longer matches
            r_host = r_host * np.float32(2.0)
            assert mem.carry_for("b", res, True, k)[1] is False
        if step == 3:
            mem.residuals["b"] = res.clone()   # replaced: a different tensor
            assert mem.carry_for("b", mem.residuals["b"], True, k)[1] is False
        if step in (1, 4):
            assert mem.carry_for("b", res, True, k)[1] is True
        out = comm.step(torch.from_numpy(g0).to(DEV), "b")
        t = g0 if r_host is None else r_host + g0
        ov, oi = O.topk_select(t, k)
        sel = np.zeros(n, dtype=bool)
        sel[oi] = True
        exp_o = np.zeros_like(t)
        exp_o[sel] = np.float32(0.0) + t[sel]
        assert same_bits(_np(out), exp_o), step
        r_host = t.copy()
        r_host[sel] = t[sel] - t[sel]
        assert same_bits(_np(mem.residuals["b"]), r_host), step


def test_short_carry_refused():
    from grace_amd import ops
    from grace_amd._lib import GraceNativeError
    n = 1 << 25
    k = O.ratio_k(n, 0.01)
    g = torch.randn(n, device=DEV)
    with pytest.raises(GraceNativeError):
        ops.topk_residual_step(g, torch.empty_like(g), False, 1.0, 1.0, k, carry=torch.empty(1000, device=DEV))


def test_carry_size_zero_where_no_bracket():
    from grace_amd import ops
    assert ops.topk_carry_size(1000, 10) == 0            # single-workgroup path
    assert ops.topk_carry_size(1 << 20, 1 << 20) == 0    # k >= n: everything selected
    assert ops.topk_carry_size(1 << 22, 41943) == 0      # stratum 32 < 256: no carry
    assert ops.topk_carry_size(1 << 25, 335544) == SAMPLE_MAX + 2


def test_carry_same_bracket_as_plain_on_repeated_gradients():
    """Three buckets whose gradients repeat every step (error feedback piles |t| up at the
    threshold): the carry path must see the same samples as the plain path, so the same fallback
    decisions, and identical results, step after step."""
    from grace_amd import ops
    n = 1 << 25
    k = O.ratio_k(n, 0.01)
    gs = [torch.randn(n, device=DEV, generator=torch.Generator(device=DEV).manual_seed(j)) for j in range(3)]
    rp = [torch.empty(n, device=DEV) for _ in range(3)]
    rc = [torch.empty(n, device=DEV) for _ in range(3)]
    cs = [torch.empty(ops.topk_carry_size(n, k), device=DEV) for _ in range(3)]
    for step in range(12):
        j = step % 3
        first = step < 3
        op, oc = torch.empty(n, device=DEV), torch.empty(n, device=DEV)
        _, vp, ip = ops.topk_residual_step(gs[j], rp[j], not first, 1.0, 1.0, k, out=op)
        st_p = ops.topk_status(n, k, gs[j].device)
        _, vc, ic = ops.topk_residual_step(gs[j], rc[j], not first, 1.0, 1.0, k, out=oc, carry=cs[j],
                                           carry_valid=not first)
        st_c = ops.topk_status(n, k, gs[j].device)
        assert st_p == st_c, (step, st_p, st_c)
        assert torch.equal(rp[j].view(torch.int32), rc[j].view(torch.int32)), step
        assert torch.equal(op.view(torch.int32), oc.view(torch.int32)), step
        assert torch.equal(torch.sort(ip).values, torch.sort(ic).values), step


def test_carry_threshold_recorded_by_parallel_fallback():
    """A mostly-zero bucket forces the parallel exact fallback (ties at 0 taken lowest index
    first): the finalize must still leave the exact threshold in the carry, and the next step with
    that carry must be exact."""
    from grace_amd import ops
    n = 1 << 25
    k = O.ratio_k(n, 0.01)
    rng = np.random.default_rng(21)
    g0 = np.zeros(n, dtype=np.float32)
    p = rng.choice(n, size=n // 400, replace=False)
    g0[p] = rng.standard_normal(p.size).astype(np.float32)
    g = torch.from_numpy(g0).to(DEV)
    res = torch.empty(n, device=DEV)
    carry = torch.empty(ops.topk_carry_size(n, k), device=DEV)
    out = torch.empty_like(g)
    _, vals, idx = ops.topk_residual_step(g, res, False, 1.0, 1.0, k, out=out, carry=carry)
    torch.cuda.synchronize()
    assert ops.topk_status(n, k, g.device) == 1
    r_host, t = _check_step(g0, None, k, vals, idx, res, out)
    c = _np(carry)
    pos = sample_positions(n)
    T = int(c[SAMPLE_MAX:].view(np.uint64)[0])
    key = t.view(np.uint32).astype(np.uint64) & np.uint64(0x7FFFFFFF)
    comp = (key << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.arange(n, dtype=np.uint64))
    assert np.count_nonzero(comp >= np.uint64(T)) == k
    assert same_bits(r_host[pos], _carried_residual(c[:SAMPLE_MAX], pos, T))
    g1 = rng.standard_normal(n, dtype=np.float32)
    _, vals, idx = ops.topk_residual_step(torch.from_numpy(g1).to(DEV), res, True, 1.0, 1.0, k, out=out,
                                          carry=carry, carry_valid=True)
    torch.cuda.synchronize()
    _check_step(g1, r_host, k, vals, idx, res, out)
