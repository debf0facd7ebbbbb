"""GPU parity of the HIP top-k engine (grace_amd/csrc/topk.hip) against the oracle and the
reference's golden vectors.  Index sets and payload values are bit-exact (the oracle uses the same
deterministic tie rule); against the reference they agree modulo ties at the k-th magnitude."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits, topk_sets_match

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _np(t):
    return t.detach().cpu().numpy()


def _sorted_payload(vals, idx):
    v, i = _np(vals), _np(idx).astype(np.int64)
    o = np.argsort(i, kind="stable")
    return v[o], i[o]


def check_topk(x_np, k, vals, idx):
    ov, oi = O.topk_select(x_np, k)
    v, i = _sorted_payload(vals, idx)
    assert i.size == k
    assert np.array_equal(i, oi.astype(np.int64)), "index set differs from oracle"
    assert same_bits(v, ov), "payload values differ from oracle"


def test_topk_golden_single(golden):
    from grace_amd.dist.compressor.topk import TopKCompressor
    for c in golden.cases("sparse", codec="topk", prefix="topk_"):
        if "steps" in c.meta:
            continue
        x = c["x"]
        ratio = c.meta["ratio"]
        comp = TopKCompressor(ratio)
        xt = torch.from_numpy(x).to(DEV)
        (vals, idx), ctx = comp.compress(xt, "w")
        assert ctx == xt.size()
        k = O.ratio_k(x.size, ratio)
        check_topk(x.ravel(), k, vals, idx)
        assert topk_sets_match(x.ravel(), _np(idx), c["idx"], k), c.name
        dec = _np(comp.decompress([vals, idx], ctx))
        assert same_bits(dec.ravel(), O.sparse_decode(*O.topk_select(x.ravel(), k), x.size)), c.name
        if np.array_equal(np.sort(_np(idx)), np.sort(c["idx"])):
            assert same_bits(dec, c["dec"]), c.name


@pytest.mark.parametrize("fused", [True, False])
def test_topk_residual_golden_sequence(golden, fused):
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    for c in golden.cases("sparse", codec="topk"):
        if "steps" not in c.meta:
            continue
        comm = Allgather(TopKCompressor(c.meta["ratio"]), ResidualMemory(), 1)
        for s in range(c.meta["steps"]):
            g = torch.from_numpy(c[f"g{s}"]).to(DEV)
            if fused:
                out = comm.step(g, "bucket")
            else:
                t = comm.memory.compensate(g, "bucket")
                payload, ctx = comm.compressor.compress(t, "bucket")
                comm.memory.update(t, "bucket", comm.compressor, payload, ctx)
                out = comm.send_receive(payload, "bucket", ctx)
            torch.cuda.synchronize()
            assert same_bits(_np(out), c[f"out{s}"]), (c.name, s, fused)
            assert same_bits(_np(comm.memory.residuals["bucket"]).ravel(), c[f"res{s}"].ravel()), (c.name, s)


def _inputs(n, kind, seed):
    g = np.random.default_rng(seed)
    if kind == "normal":
        return g.standard_normal(n).astype(np.float32)
    if kind == "ties":
        return (np.round(g.standard_normal(n) * 4) / 4).astype(np.float32)
    if kind == "ramp":          # sorted magnitudes: the largest values are clustered at the end
        return np.linspace(-1, 3, n, dtype=np.float32)
    if kind == "sparse":        # mostly zeros: forces the exact fallback when k > nnz
        x = np.zeros(n, dtype=np.float32)
        pos = g.choice(n, size=max(1, n // 400), replace=False)
        x[pos] = g.standard_normal(pos.size).astype(np.float32)
        return x
    if kind == "special":
        x = g.standard_normal(n).astype(np.float32)
        x[g.choice(n, 5, replace=False)] = np.nan
        x[g.choice(n, 5, replace=False)] = np.inf
        x[g.choice(n, 5, replace=False)] = -np.inf
        x[g.choice(n, 50, replace=False)] = -0.0
        return x
    if kind == "scaled":        # heavy-tailed magnitudes spanning many octaves
        return (g.standard_normal(n) * np.exp(g.standard_normal(n) * 3)).astype(np.float32)
    raise ValueError(kind)


@pytest.mark.parametrize("n", [32768, 32769, 100003, 1 << 20, (1 << 22) + 77])
@pytest.mark.parametrize("ratio", [0.01, 0.001, 0.3])
@pytest.mark.parametrize("kind", ["normal", "ties", "ramp", "sparse", "special", "scaled"])
def test_topk_compress_vs_oracle(n, ratio, kind):
    from grace_amd import ops
    x = _inputs(n, kind, seed=n + int(ratio * 1e4))
    k = O.ratio_k(n, ratio)
    _, vals, idx = ops.topk_compress(torch.from_numpy(x).to(DEV), k)
    check_topk(x, k, vals, idx)


@pytest.mark.parametrize("n", [40000, (1 << 21) + 5])
@pytest.mark.parametrize("kind", ["normal", "sparse", "special"])
@pytest.mark.parametrize("with_out", [True, False])
def test_topk_residual_step_vs_oracle(n, kind, with_out):
    from grace_amd import ops
    k = O.ratio_k(n, 0.01)
    g0 = _inputs(n, kind, 1)
    r0 = (0.1 * _inputs(n, "normal", 2)).astype(np.float32)
    g, r = torch.from_numpy(g0).to(DEV), torch.from_numpy(r0).to(DEV)
    out = torch.empty_like(g) if with_out else None
    _, vals, idx = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    t, ov, oi, ores, oout = O.topk_residual_step(g0, r0, 0.01)
    check_topk(t, k, vals, idx)
    assert same_bits(_np(r), ores)
    if with_out:
        assert same_bits(_np(out), oout)


@pytest.mark.parametrize("n", [1000, 32768, 32769, 100003, (1 << 21) + 5])
@pytest.mark.parametrize("kind", ["normal", "ties", "sparse", "special"])
def test_topk_nomemory_step_one_pass(n, kind):
    """Allgather(TopK, NoneMemory).step at world 1 through the one-pass path (grace_topk_step_dense):
    payload and (0 + decode) / 1 bit-exact against the oracle's compress + decompress + Python sum;
    the input is left untouched.  'sparse' takes the exact fallback (k > non-zeros)."""
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.none import NoneMemory
    x = _inputs(n, kind, seed=n + 3)
    xt = torch.from_numpy(x).to(DEV)
    k = O.ratio_k(n, 0.01)
    expect = np.float32(0.0) + O.sparse_decode(*O.topk_select(x, k), n)     # Python sum starts at 0
    _, vals, idx, out = ops.topk_step_dense(xt, k)
    check_topk(x, k, vals, idx)
    assert same_bits(_np(out), expect)
    comm = Allgather(TopKCompressor(0.01), NoneMemory(), 1)
    out2 = comm.step(xt.view(-1, 1) if n % 2 else xt, "w")
    assert tuple(out2.shape) == ((n, 1) if n % 2 else (n,))
    assert same_bits(_np(out2).ravel(), expect)
    assert same_bits(_np(xt), x)


def test_topk_fallback_taken_and_exact():
    """k larger than the number of non-zeros: the sampled bracket cannot hold; the exact
    single-workgroup path must produce the oracle's result (lowest-index zeros fill the tail)."""
    from grace_amd import ops
    n = 1 << 20
    x = _inputs(n, "sparse", 7)
    k = O.ratio_k(n, 0.01)
    xt = torch.from_numpy(x).to(DEV)
    _, vals, idx = ops.topk_compress(xt, k)
    assert ops.topk_status(n, k, xt.device) == 1
    check_topk(x, k, vals, idx)
    # a normal input takes the fast path
    y = _inputs(n, "normal", 8)
    _, vals, idx = ops.topk_compress(torch.from_numpy(y).to(DEV), k)
    assert ops.topk_status(n, k, xt.device) == 0
    check_topk(y, k, vals, idx)


def test_topk_full_bucket_256mib():
    """BASELINE config: top-k 1 % + residual on a 256 MiB bucket, exact against the oracle."""
    from grace_amd import ops
    n = 64 * 1024 * 1024
    k = O.ratio_k(n, 0.01)
    gen = torch.Generator(device="cpu").manual_seed(1)
    g_cpu = torch.randn(n, generator=gen)
    r_cpu = 0.1 * torch.randn(n, generator=torch.Generator().manual_seed(2))
    g, r = g_cpu.to(DEV), r_cpu.to(DEV)
    out = torch.empty_like(g)
    _, vals, idx = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    torch.cuda.synchronize()
    assert ops.topk_status(n, k, g.device) == 0
    t = (r_cpu + g_cpu).numpy()
    ov, oi = O.topk_select(t, k)
    v, i = _sorted_payload(vals, idx)
    assert np.array_equal(i, oi.astype(np.int64))
    assert same_bits(v, ov)
    res = _np(r)
    sel = np.zeros(n, dtype=bool)
    sel[oi] = True
    assert same_bits(res[~sel], t[~sel]) and not np.any(res[sel])
    o = _np(out)
    assert same_bits(o[sel], t[sel]) and not np.any(o[~sel])


def test_topk_parallel_fallback_sparse_256mib():
    """A 256 MiB bucket that is 99.75 % exact zeros (k = 1 % > non-zeros: massive ties at 0, so the
    candidate list overflows): the parallel exact fallback (all finalize workgroups, grid barriers)
    must give the oracle's result -- every non-zero plus the lowest-index zeros -- in milliseconds,
    not the single-workgroup path's ~150 ms."""
    from grace_amd import ops
    n = 64 * 1024 * 1024
    k = O.ratio_k(n, 0.01)
    rng = np.random.default_rng(11)
    g0 = np.zeros(n, dtype=np.float32)
    pos = rng.choice(n, size=n // 400, replace=False)
    g0[pos] = rng.standard_normal(pos.size).astype(np.float32)
    r0 = np.zeros(n, dtype=np.float32)
    g, r = torch.from_numpy(g0).to(DEV), torch.from_numpy(r0).to(DEV)
    out = torch.empty_like(g)
    ops.topk_residual_step(g, r.clone(), True, 1.0, 1.0, k, out=torch.empty_like(g))   # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _, vals, idx = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    e1.record()
    torch.cuda.synchronize()
    assert ops.topk_status(n, k, g.device) == 1
    assert e0.elapsed_time(e1) < 30.0, e0.elapsed_time(e1)
    ov, oi = O.topk_select(g0, k)
    v, i = _sorted_payload(vals, idx)
    assert np.array_equal(i, oi.astype(np.int64))
    assert same_bits(v, ov)
    sel = np.zeros(n, dtype=bool)
    sel[oi] = True
    res, o = _np(r), _np(out)
    assert same_bits(res[~sel], g0[~sel]) and not np.any(res[sel])
    assert same_bits(o[sel], g0[sel]) and not np.any(o[~sel])


@pytest.mark.parametrize("n,offset", [(70001, 0), (100003, 1), ((1 << 22) + 5, 0), ((1 << 22) + 7, 3)])
def test_topk_parallel_fallback_slices(n, offset):
    """The claimed-slice parallel fallback (csrc/topk.hip parallel_exact) at sizes whose slices do
    not tile the bucket, on 16-B aligned and unaligned views (scalar path), with the ties at the
    k-th key (zeros) spread over every slice: bit-exact against the oracle, residual and output too."""
    from grace_amd import ops
    rng = np.random.default_rng(n + offset)
    base = np.zeros(n + offset, dtype=np.float32)
    nz = rng.choice(n, size=n // 300, replace=False) + offset
    base[nz] = rng.standard_normal(nz.size).astype(np.float32)
    base[offset + rng.choice(n, size=n // 400, replace=False)] = 0.5   # ties above the cut
    x = base[offset:]
    k = O.ratio_k(n, 0.01)                   # > the non-zeros: the cut is at key 0, tied everywhere
    buf = torch.from_numpy(base).to(DEV)
    g = buf[offset:]
    rbuf = torch.zeros(n + offset, device=DEV)
    r = rbuf[offset:]
    obuf = torch.empty(n + offset, device=DEV)
    out = obuf[offset:]
    _, vals, idx = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    torch.cuda.synchronize()
    assert ops.topk_status(n, k, g.device) == 1
    ov, oi = O.topk_select(x, k)
    v, i = _sorted_payload(vals, idx)
    assert np.array_equal(i, oi.astype(np.int64))
    assert same_bits(v, ov)
    sel = np.zeros(n, dtype=bool)
    sel[oi] = True
    res, o = _np(r), _np(out)
    assert same_bits(res[~sel], x[~sel]) and not np.any(res[sel])
    assert same_bits(o[sel], x[sel]) and not np.any(o[~sel])


def test_topk_fallback_runout_raises():
    """a wait of the parallel exact fallback that runs out must never pass as a
    result.  With the wait bound forced to 0 polls, the sparse step (fallback taken) aborts: the
    device status reads 2, the next top-k call raises TopKWaitError, and TopKCompressor with
    check_sync=True raises on the failing call itself.  With the bound restored, the fallback's
    scratch (re-zeroed by the last workgroup out, also after an abort) gives exact results again."""
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n = 1 << 22
    k = O.ratio_k(n, 0.01)
    rng = np.random.default_rng(5)
    g0 = np.zeros(n, dtype=np.float32)
    pos = rng.choice(n, size=n // 400, replace=False)
    g0[pos] = rng.standard_normal(pos.size).astype(np.float32)
    g = torch.from_numpy(g0).to(DEV)
    ops.topk_check()                         # nothing pending from earlier tests
    prev = ops.topk_fallback_spin_limit(0)
    try:
        ops.topk_residual_step(g, torch.zeros_like(g), True, 1.0, 1.0, k, out=torch.empty_like(g))
        torch.cuda.synchronize()
        assert ops.topk_status(n, k, g.device) == 2
        with pytest.raises(ops.TopKWaitError):
            ops.topk_compress(g, k)          # the next call reports the earlier abort
        comm = Allgather(TopKCompressor(0.01, check_sync=True), ResidualMemory(), 1)
        with pytest.raises(ops.TopKWaitError):
            comm.step(g, "w")                # check_sync: the failing call itself raises
    finally:
        ops.topk_fallback_spin_limit(prev)
    assert ops.topk_fallback_spin_limit() == prev
    torch.cuda.synchronize()
    ops._topk_status()                       # the word was taken by the raise: nothing pending
    r = torch.zeros_like(g)
    out = torch.empty_like(g)
    _, vals, idx = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=out)
    ops.topk_check()
    assert ops.topk_status(n, k, g.device) == 1
    check_topk(g0, k, vals, idx)
    ov, oi = O.topk_select(g0, k)
    sel = np.zeros(n, dtype=bool)
    sel[oi] = True
    o = _np(out)
    assert same_bits(o[sel], g0[sel]) and not np.any(o[~sel])


@pytest.mark.parametrize("n,case", [(1 << 22, "normal"), ((1 << 22) + 3, "normal"), (1 << 22, "sparse"),
                                    (20000, "normal"), (100003, "ties"), ((1 << 20) + 1, "special")])
def test_topk_residual_step_swap_equals_in_place(n, case):
    """The world > 1 step into a second residual buffer (grace_topk_residual_step_swap: provisional
    picks zeroed in the main pass, finalize fix-ups from t = g + r_in) leaves exactly the residual
    and payload of the in-place step, over a 3-step chain (first step without a residual, then
    with), including the exact fallback (sparse) and the single-workgroup path (n <= 32768);
    r_in is never written."""
    from grace_amd import ops
    k = O.ratio_k(n, 0.01)
    r_a = torch.zeros(n, device=DEV)              # in place
    r_b = [torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)]
    for step in range(3):
        g0 = _inputs(n, case, 40 + step)
        g = torch.from_numpy(g0).to(DEV)
        _, va, ia = ops.topk_residual_step(g, r_a, step > 0, 1.0, 1.0, k, out=None)
        r_in, r_out = r_b[step % 2], r_b[(step + 1) % 2]
        before = r_in.clone()
        _, vb, ib = ops.topk_residual_step_swap(g, r_in, step > 0, 1.0, 1.0, k, r_out)
        torch.cuda.synchronize()
        assert same_bits(_np(r_in), _np(before)), "r_in was written"
        assert same_bits(_np(r_out), _np(r_a)), (step, "residual differs")
        sa, sb = _sorted_payload(va, ia), _sorted_payload(vb, ib)
        assert np.array_equal(sa[1], sb[1]) and same_bits(sa[0], sb[0]), (step, "payload differs")
