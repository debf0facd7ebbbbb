"""GPU parity of the one-pass world-1 PowerSGD compress (grace_powersgd_w1_compress: psgd_w1_pass +
psgd_w1_fin in grace_amd/csrc/powersgd.hip) against an f64 restatement of the reference algorithm
(grace_dl/dist/compressor/powersgd.py:40-56 at world size 1: P = orthogonalize(M q), Q = M^T P),
within the f32 tolerance rel <= 1e-5 * sqrt(m) of SURVEY.md §8a, plus the robust (ill-conditioned)
path and the workspace contract (counters left zero, shapes sharing one workspace)."""
import numpy as np
import pytest
import torch

from grace_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def _exact_qr(a):
    q, r = np.linalg.qr(np.asarray(a, dtype=np.float64))
    return q * np.where(np.diag(r) < 0, -1.0, 1.0)


def _expect(M, q):
    """f64 reference: P = QR factor of M q (Gram-Schmidt signs), Q = M^T P."""
    P = _exact_qr(M.astype(np.float64) @ q.astype(np.float64))
    return P, M.T.astype(np.float64) @ P


def _close(a, b, m, scale=None):
    tol = 1e-5 * np.sqrt(m)
    scale = np.abs(b).max() if scale is None else scale
    return np.allclose(a, b, rtol=tol, atol=tol * max(scale, 1e-30))


def _counters_zero():
    """Arrival / read counters and the run-out count left zero.  Word 0 is the robust path's flag:
    it keeps the tag of the last call that set it (each call waits for its own tag), so it is not
    a counter and is not reset."""
    ws = ops.workspace("powersgd_w1", 256, torch.device(DEV))
    head = _np(ws[: 256 + 2 * 4 * 16384].view(torch.int32))
    return not head[1:].any()


@pytest.mark.parametrize("shape", [(4096, 4096), (256, 300), (100, 1000), (4097, 1028), (64, 16384), (9000, 256),
                                   (20000, 4096), (1, 8), (65, 4)])
@pytest.mark.parametrize("drawn", [False, True])
def test_w1_compress_vs_f64(shape, drawn):
    n, m = shape
    rng = np.random.default_rng(n * 7 + m)
    M = rng.standard_normal(shape).astype(np.float32)
    Md = _t(M)
    if n < 4:
        pytest.skip("rank 4 needs n >= 4")
    assert ops.powersgd_w1_ok(Md, 4)
    if drawn:
        seed = 99 + n
        P, Q = ops.powersgd_w1_compress(Md, seed=seed)
        q = _np(ops.normal((m, 4), seed, DEV))
    else:
        q = rng.standard_normal((m, 4)).astype(np.float32)
        P, Q = ops.powersgd_w1_compress(Md, q=_t(q))
    Pe, Qe = _expect(M, q)
    assert np.isfinite(_np(P)).all() and np.isfinite(_np(Q)).all()
    assert _close(_np(P), Pe, m, scale=1.0), np.abs(_np(P) - Pe).max()
    assert _close(_np(Q), Qe, n), np.abs(_np(Q) - Qe).max() / np.abs(Qe).max()
    assert _counters_zero()


def test_w1_matches_separate_kernels():
    """Same (P, Q) as the unfused sequence powersgd_p -> orthogonalize -> powersgd_qt, within the
    f32 tolerance (the fused Q is the more accurate: f64 Qraw)."""
    rng = np.random.default_rng(3)
    M = rng.standard_normal((4096, 4096)).astype(np.float32)
    q = rng.standard_normal((4096, 4)).astype(np.float32)
    Md, qd = _t(M), _t(q)
    P1, Q1 = ops.powersgd_w1_compress(Md, q=qd)
    P2 = ops.orthogonalize_(ops.powersgd_p(Md, qd))
    Q2 = ops.powersgd_qt(Md, P2)
    assert _close(_np(P1), _np(P2), 4096, scale=1.0)
    assert _close(_np(Q1), _np(Q2), 4096)


@pytest.mark.parametrize("n,m,rank", [(4096, 4096, 2), (3000, 2048, 3), (9000, 1024, 1)])
def test_w1_ill_conditioned_robust_path(n, m, rank):
    """M of rank < 4 makes P_raw = M q rank-deficient: the Cholesky pivots fail, workgroup 0
    orthogonalises P_raw by MGS2 and publishes it, and every workgroup computes Q = M^T P directly.
    P finite with orthonormal (or exactly zero) columns, Q = M^T P to f32 accuracy; the leading
    `rank` columns are the exact factor."""
    rng = np.random.default_rng(n + rank)
    M = (rng.standard_normal((n, rank)) @ rng.standard_normal((rank, m))).astype(np.float32)
    q = rng.standard_normal((m, 4)).astype(np.float32)
    P, Q = ops.powersgd_w1_compress(_t(M), q=_t(q))
    P, Q = _np(P), _np(Q)
    assert np.isfinite(P).all() and np.isfinite(Q).all()
    Pr = M.astype(np.float64) @ q.astype(np.float64)
    assert np.abs(P[:, :rank] - _exact_qr(Pr[:, :rank])).max() < 1e-4
    G = P.T.astype(np.float64) @ P
    for c in range(4):
        if np.abs(P[:, c]).max() > 0:
            assert abs(G[c, c] - 1.0) < 1e-4
    Qe = M.T.astype(np.float64) @ P.astype(np.float64)
    assert np.abs(Q - Qe).max() <= 1e-5 * np.sqrt(n) * np.abs(Qe).max()
    assert _counters_zero()


def test_w1_shapes_share_one_workspace():
    """Big, small, big again on the same workspace: the fixed-offset counters stay zero and every
    call's result is unaffected by the previous call's shape."""
    rng = np.random.default_rng(11)
    shapes = [(4096, 4096), (128, 64), (20000, 4096), (300, 8192), (4096, 4096)]
    Ms = [rng.standard_normal(s).astype(np.float32) for s in shapes[:4]]
    qs = [rng.standard_normal((s[1], 4)).astype(np.float32) for s in shapes[:4]]
    Ms.append(Ms[0])
    qs.append(qs[0])
    outs = [tuple(map(_np, ops.powersgd_w1_compress(_t(M), q=_t(q)))) for M, q in zip(Ms, qs)]
    assert np.array_equal(outs[0][0], outs[4][0]) and np.array_equal(outs[0][1], outs[4][1])
    for (P, Q), M, q in zip(outs, Ms, qs):
        Pe, Qe = _expect(M, q)
        assert _close(P, Pe, M.shape[1], scale=1.0)
        assert _close(Q, Qe, M.shape[0])
    assert _counters_zero()


def test_w1_deterministic():
    rng = np.random.default_rng(12)
    Md = _t(rng.standard_normal((4096, 4096)).astype(np.float32))
    a = [tuple(map(_np, ops.powersgd_w1_compress(Md, seed=5))) for _ in range(3)]
    assert all(np.array_equal(a[0][i], x[i]) for x in a[1:] for i in range(2))


def test_compressor_takes_the_w1_path_and_matches_reference_algorithm():
    """PowerSGDCompressor(rank=4) at world size 1 runs the one-pass kernels (the unfused launch
    sequence is not used) and returns the reference's (P, Q) on the device draw."""
    from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
    rng = np.random.default_rng(13)
    M = rng.standard_normal((1024, 2048)).astype(np.float32)
    comp = PowerSGDCompressor(rank=4)
    called = {}
    orig = ops.powersgd_qt
    ops.powersgd_qt = lambda *a, **k: called.setdefault("qt", orig(*a, **k))
    try:
        _, (p, q, _) = comp.compress(_t(M), "w")
    finally:
        ops.powersgd_qt = orig
    assert "qt" not in called
    q0 = _np(ops.normal((2048, 4), ops.step_seed("powersgd-q", "w", 1), DEV))
    Pe, Qe = _expect(M, q0)
    assert _close(_np(p), Pe, 2048, scale=1.0)
    assert _close(_np(q), Qe, 1024)


def test_w1_two_streams_ordered_and_exact():
    """two one-pass compresses issued on two streams at once.  Their grids (one
    workgroup per CU, spinning exchanges) must never run concurrently: ops orders a call on a new
    stream behind the previous call's stream.  Both results equal the one-stream results bit for
    bit, and the status word reports no wait that ran out."""
    rng = np.random.default_rng(31)
    Ms = [_t(rng.standard_normal((4096, 4096)).astype(np.float32)) for _ in range(4)]
    qs = [_t(rng.standard_normal((4096, 4)).astype(np.float32)) for _ in range(4)]
    ref = [tuple(_np(x) for x in ops.powersgd_w1_compress(M, q)) for M, q in zip(Ms, qs)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for rep in range(3):
        for j, (M, q) in enumerate(zip(Ms, qs)):
            with torch.cuda.stream(streams[j % 2]):
                outs.append((j, ops.powersgd_w1_compress(M, q)))
    torch.cuda.synchronize()
    for j, (P, Q) in outs:
        assert np.array_equal(_np(P), ref[j][0]) and np.array_equal(_np(Q), ref[j][1]), j
    ops.powersgd_w1_check()              # raises if any wait ran out
    assert _counters_zero()


def test_w1_status_word_raises():
    """A wait that ran out (status bit 1, written by the kernels into the pinned word) makes the
    next call raise instead of returning silently wrong P / Q."""
    M = _t(np.random.default_rng(2).standard_normal((512, 256)).astype(np.float32))
    ops.powersgd_w1_compress(M)
    torch.cuda.synchronize()
    st, view = ops._w1_st[str(M.device)]
    view[0] = 2
    with pytest.raises(ops.PowerSGDWaitError):
        ops.powersgd_w1_compress(M)
    assert int(view[0]) == 0
    ops.powersgd_w1_compress(M)          # cleared: the next call runs
    ops.powersgd_w1_check()
