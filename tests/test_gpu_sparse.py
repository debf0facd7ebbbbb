"""GPU parity of random-k and threshold (grace_amd/csrc/sparse.hip) against golden vectors."""
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


def test_randomk_golden_torch_rng(golden):
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    for c in golden.cases("sparse", codec="randomk"):
        if "steps" in c.meta:
            continue
        comp = RandomKCompressor(c.meta["ratio"], rng="torch_cpu")
        comp.global_step = c.meta["seed"] - sum(bytes(c.meta["name"], encoding="utf8"))
        (vals,), ctx = comp.compress(_t(c["x"]), c.meta["name"])
        assert np.array_equal(_np(ctx[0]), c["idx"]), c.name
        assert same_bits(_np(vals), c["vals"]), c.name
        assert same_bits(_np(comp.decompress([vals], ctx)), c["dec"]), c.name


def test_randomk_device_rng_properties():
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    x = np.random.default_rng(0).standard_normal(100003).astype(np.float32)
    a, b = RandomKCompressor(0.01), RandomKCompressor(0.01)
    (va,), ca = a.compress(_t(x), "layer.w")
    (vb,), cb = b.compress(_t(x), "layer.w")
    idx = _np(ca[0])
    assert idx.size == 1000 and idx.min() >= 0 and idx.max() < x.size
    assert np.array_equal(idx, _np(cb[0]))                      # same seed on every rank
    assert same_bits(_np(va), x[idx])
    (vc,), cc = a.compress(_t(x), "layer.w")                     # next step: new indices
    assert not np.array_equal(idx, _np(cc[0]))
    dec = _np(a.decompress([va], ca))
    assert same_bits(dec, O.randomk_decode(x[idx], idx, x.size))


def test_randomk_allreduce_residual_sequence(golden):
    from grace_amd.dist.communicator.allreduce import Allreduce
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    c = golden.case("sparse", "randomk_residual_allreduce")
    comm = Allreduce(RandomKCompressor(0.1, rng="torch_cpu"), ResidualMemory(), 1)
    for s in range(2):
        out = comm.step(_t(c[f"g{s}"]), "w")
        assert same_bits(_np(out), c[f"out{s}"].ravel()), s
        assert same_bits(_np(comm.memory.residuals["w"]).ravel(), c[f"res{s}"].ravel()), s


def test_threshold_golden(golden):
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    for c in golden.cases("sparse", codec="threshold"):
        comp = ThresholdCompressor(c.meta["threshold"])
        (vals, idx), ctx = comp.compress(_t(c["x"]), "w")
        assert np.array_equal(_np(idx), c["idx"]), c.name
        assert same_bits(_np(vals), c["vals"]), c.name
        assert same_bits(_np(comp.decompress([vals, idx], ctx)), c["dec"]), c.name


@pytest.mark.parametrize("n", [1, 5000, 16384, 16385, 1 << 20])
@pytest.mark.parametrize("thr", [0.01, 1.0, 3.0, 1e9])
def test_threshold_vs_oracle(n, thr):
    x = np.random.default_rng(n).standard_normal(n).astype(np.float32)
    vals, idx = ops.threshold_compress(_t(x), thr)
    ov, oi = O.threshold_select(x, thr)
    assert np.array_equal(_np(idx), oi)
    assert same_bits(_np(vals), ov)


def test_threshold_nan_max_uses_threshold():
    x = np.array([0.5, np.nan, -2.0, 0.01, 3.0], dtype=np.float32)
    vals, idx = ops.threshold_compress(_t(x), 1.0)
    ov, oi = O.threshold_select(x, 1.0)
    assert np.array_equal(_np(idx), oi)


def test_threshold_allgather_world1_variable_path():
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    x = np.random.default_rng(9).standard_normal(20000).astype(np.float32)
    comm = Allgather(ThresholdCompressor(1.5), ResidualMemory(), 1)
    out = _np(comm.step(_t(x), "w"))
    ov, oi = O.threshold_select(x, 1.5)
    exp = (O.python_sum([O.sparse_decode(ov, oi, x.size)]) / np.float32(1)).astype(np.float32)
    assert same_bits(out, exp)
    res = _np(comm.memory.residuals["w"])
    assert same_bits(res, O.residual_update(x, O.sparse_decode(ov, oi, x.size)))


@pytest.mark.parametrize("n", [1, 5000, 16385, 1 << 20])
@pytest.mark.parametrize("thr", [0.01, 1.5, 1e9])
@pytest.mark.parametrize("memory", ["none", "residual"])
def test_threshold_fused_one_read_step_sequence(n, thr, memory):
    """threshold.fused_step (device recount, one host read): three steps bit-exact against the
    oracle's compensate -> select -> decode -> residual sequence, including thresholds above the
    signed max (recount at min(thr, max)), an all-negative step and the generic path."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    from grace_amd.dist.memory.none import NoneMemory
    from grace_amd.dist.memory.residual import ResidualMemory
    comp = ThresholdCompressor(thr)
    comm = Allgather(comp, ResidualMemory() if memory == "residual" else NoneMemory(), 1)
    assert comp.fused_step(comm, _t(np.zeros(4, np.float32)), "probe") is not None
    rng = np.random.default_rng(n + int(thr))
    res = None
    for s in range(3):
        x = rng.standard_normal(n).astype(np.float32)
        if s == 1:
            x = -np.abs(x)                                      # signed max < 0: threshold becomes max
        out = _np(comm.step(_t(x), "w"))
        t = O.residual_compensate(x, res) if memory == "residual" else x
        ov, oi = O.threshold_select(t, thr)
        dec = O.sparse_decode(ov, oi, n)
        assert same_bits(out, (O.python_sum([dec]) / np.float32(1)).astype(np.float32)), s
        if memory == "residual":
            res = O.residual_update(t, dec)
            assert same_bits(_np(comm.memory.residuals["w"]), res), s


@pytest.mark.parametrize("case", ["nan", "neg_inf_all_negative", "neg_zero", "thr_nonpositive", "big_unaligned"])
@pytest.mark.parametrize("memory", ["none", "residual"])
def test_threshold_world1_speculative_pass_special_values(case, memory):
    """The world-1 step selects at thr in one pass and fixes up at max t only when max t < thr
    (grace_threshold_step_w1): NaN (bound stays thr), -inf in an all-negative tensor (fix-up path,
    t recovered from the first pass's out / r'), signed zeros, thresholds <= 0 and a multi-chunk
    unaligned tensor, two steps each, bit-exact against the oracle sequence."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    from grace_amd.dist.memory.none import NoneMemory
    from grace_amd.dist.memory.residual import ResidualMemory
    rng = np.random.default_rng(len(case))
    n = (1 << 22) + 3 if case == "big_unaligned" else 40000
    thr = -0.5 if case == "thr_nonpositive" else 1.5
    comm = Allgather(ThresholdCompressor(thr), ResidualMemory() if memory == "residual" else NoneMemory(), 1)
    res = None
    for s in range(2):
        x = rng.standard_normal(n).astype(np.float32)
        if case == "nan":
            x[rng.choice(n, 3, replace=False)] = np.nan
            x = -np.abs(x) * np.float32(0.1)                 # max < thr, but NaN keeps the bound at thr
        elif case == "neg_inf_all_negative":
            x = -np.abs(x) - np.float32(0.25)
            x[rng.choice(n, 4, replace=False)] = -np.inf
        elif case == "neg_zero":
            x[rng.choice(n, 500, replace=False)] = -0.0
            if s == 1:
                x = -np.abs(x)
        elif case == "thr_nonpositive":
            x = -np.abs(x) - np.float32(1.0)                  # every element < thr <= 0
            x[rng.choice(n, 7, replace=False)] = -0.0 if s == 0 else -3.0
        out = _np(comm.step(_t(x), "w"))
        t = O.residual_compensate(x, res) if memory == "residual" else x
        ov, oi = O.threshold_select(t, thr)
        dec = O.sparse_decode(ov, oi, n)
        assert same_bits(out, (O.python_sum([dec]) / np.float32(1)).astype(np.float32)), (case, s)
        if memory == "residual":
            res = O.residual_update(t, dec)
            assert same_bits(_np(comm.memory.residuals["w"]), res), (case, s)


@pytest.mark.parametrize("memory", ["none", "residual"])
def test_threshold_capacity_exchange_retry_bit_exact(memory):
    """exchange='capacity', overflow='retry': the first step learns the capacity through the counts
    exchange, later steps send fixed-size records; a step whose count outgrows the capacity is redone
    exactly.  Every step bit-exact with the oracle sequence."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    from grace_amd.dist.memory.none import NoneMemory
    from grace_amd.dist.memory.residual import ResidualMemory
    n = 300_007
    comp = ThresholdCompressor(2.0, exchange="capacity", capacity_margin=1.25)
    comm = Allgather(comp, ResidualMemory() if memory == "residual" else NoneMemory(), 1)
    rng = np.random.default_rng(77)
    res = None
    scales = [1.0, 1.0, 1.05, 2.0, 1.0, 0.1]      # step 3 overflows (count grows ~8x)
    for s, sc in enumerate(scales):
        x = (rng.standard_normal(n) * sc).astype(np.float32)
        out = _np(comm.step(_t(x), "w"))
        t = O.residual_compensate(x, res) if memory == "residual" else x
        ov, oi = O.threshold_select(t, 2.0)
        dec = O.sparse_decode(ov, oi, n)
        assert same_bits(out, dec), s
        if memory == "residual":
            res = O.residual_update(t, dec)
            assert same_bits(_np(comm.memory.residuals["w"]), res), s
        assert comp.capacity["w"] >= 64
    assert comp.overflows >= 1


def test_threshold_capacity_exchange_defer_keeps_overflow_in_residual():
    """overflow='defer' (ResidualMemory): no host read in the step.  Without overflow the step is
    bit-exact; on overflow only the first `cap` selected entries (ascending index) are sent, the rest
    stay in the residual, and the next step of the name runs with a grown capacity.  Inputs: small
    noise plus c_s spikes of magnitude 5, so the selected count is controlled step by step."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n, margin = 200_003, 1.5
    comp = ThresholdCompressor(2.0, exchange="capacity", capacity_margin=margin, overflow="defer")
    comm = Allgather(comp, ResidualMemory(), 1)
    rng = np.random.default_rng(5)
    grow = lambda mx: int(min(n, max(64, int(np.ceil(mx * margin)))))
    res, cap, prev = None, None, None      # mirror of the capacity policy (threshold._settle)
    truncated = 0
    for s, c in enumerate([1000, 1000, 5000, 1000, 1000]):
        x = (rng.standard_normal(n) * 0.01).astype(np.float32)
        x[rng.choice(n, c, replace=False)] = np.float32(5.0)
        if prev is not None and (prev[0] > prev[1] or grow(prev[0]) * 4 < prev[1]):
            cap = grow(prev[0])
        out = _np(comm.step(_t(x), "w"))
        t = O.residual_compensate(x, res)
        ov, oi = O.threshold_select(t, 2.0)
        if cap is None:
            cap, prev = grow(oi.size), None                 # learned through the counts exchange
        else:
            prev = (oi.size, cap)
            if oi.size > cap:
                ov, oi = ov[:cap], oi[:cap]
                truncated += 1
        assert comp.capacity["w"] == cap or prev is not None, s
        dec = O.sparse_decode(ov, oi, n)
        res = O.residual_update(t, dec)
        assert same_bits(out, dec), s
        assert same_bits(_np(comm.memory.residuals["w"]), res), s
    assert truncated == 1
    torch.cuda.synchronize()
    comp._settle("w", n)
    assert comp.overflows == 1


@pytest.mark.parametrize("world,n,k", [(1, 4099, 40), (2, 100003, 1000), (3, (1 << 20) + 17, 20000),
                                       (8, 5_000_000, 50000)])
def test_sparse_aggregate_rank_ordered(world, n, k):
    """Allgather decode + aggregate of W top-k payloads (allgather.py:40-45): bit-exact with the
    Python sum of the dense decodes in rank order, divided by W -- with overlapping selections,
    -0.0 and NaN values, and an output length that is not a multiple of the 4096-element chunk."""
    from grace_amd import ops as G
    rng = np.random.default_rng(world * 7 + k)
    shared = rng.choice(n, k // 2, replace=False)          # indices every rank selects
    vals_l, idx_l, decs = [], [], []
    for w in range(world):
        own = rng.choice(np.setdiff1d(np.arange(n), shared), k - shared.size, replace=False)
        idx = rng.permutation(np.concatenate([shared, own])).astype(np.int32)
        v = rng.standard_normal(k).astype(np.float32)
        v[:5] = np.float32(-0.0)
        v[5] = np.nan
        vals_l.append(v)
        idx_l.append(idx)
        decs.append(O.sparse_decode(v, idx, n))
    payload = np.concatenate([np.concatenate([v, i.view(np.float32)]) for v, i in zip(vals_l, idx_l)])
    buf = _t(payload)
    # chunk-grouped payloads (grace_sort_payload) for the one-pass aggregate
    sorted_buf = torch.cat([G.sort_payload(buf[w * 2 * k:(w + 1) * 2 * k], k, n) for w in range(world)])
    L = ops.sorted_payload_len(k, n)
    nch, ow = (n + 8191) // 8192, (k + 1) // 2
    assert L == k + ow + nch                                          # 6 B per entry + the chunk ends
    for w in range(world):
        base = w * L
        vals_s = _np(sorted_buf[base:base + k])
        offs = _np(sorted_buf[base + k:base + k + ow].view(torch.int16)).view(np.uint16)[:k].astype(np.int64)
        ends = _np(sorted_buf[base + k + ow:base + L].view(torch.int32))
        assert ends.size == nch and ends[-1] == k and np.all(np.diff(ends) >= 0)
        assert np.all(offs < 8192)
        idx_s = np.searchsorted(ends, np.arange(k), side="right") * 8192 + offs   # grouped by 8192-chunk
        order = np.argsort(idx_s)
        assert np.array_equal(idx_s[order], np.sort(idx_l[w]))        # same entries
        assert same_bits(vals_s[order], vals_l[w][np.argsort(idx_l[w])])
    for divisor in (world, 1):
        out = _np(G.sparse_aggregate(buf, buf[k:].view(torch.int32), 2 * k, [k] * world, world, n, divisor))
        exp = O.python_sum(decs)
        if divisor != 1:
            exp = (exp / np.float32(divisor)).astype(np.float32)
        assert same_bits(out, exp), (world, divisor)
        out2 = _np(G.sparse_aggregate_sorted(sorted_buf, k, world, n, divisor))
        assert same_bits(out2, exp), ("sorted", world, divisor)


def test_sort_payload_workspace_reuse_across_sizes():
    """grace_sort_payload's arrival ticket sits at a fixed place in the shared workspace: a small-n
    call after a large-n call (whose chunk counts filled the workspace) must still group correctly."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    for n, k in ((1 << 24, 20000), (100000, 1000), (1 << 24, 20000), (50000, 700)):
        idx = rng.choice(n, size=k, replace=False).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        buf = torch.cat([torch.from_numpy(vals), torch.from_numpy(idx.view(np.float32))]).to(dev)
        out = ops.sort_payload(buf, k, n).cpu().numpy()
        ow = (k + 1) // 2
        ov = out[:k]
        offs = out[k:k + ow].view(np.uint16)[:k].astype(np.int64)
        ends = out[k + ow:].view(np.int32)
        assert ends[-1] == k and np.all(np.diff(ends) >= 0), (n, k)
        oi = np.searchsorted(ends, np.arange(k), side="right") * 8192 + offs
        order = np.argsort(idx)
        o2 = np.argsort(oi)
        assert np.array_equal(idx[order], oi[o2]) and np.array_equal(vals[order], ov[o2]), (n, k)


@pytest.mark.parametrize("n", [1000, 4097, (1 << 20) + 3])
@pytest.mark.parametrize("rng", ["device", "torch_cpu"])
def test_randomk_world1_fused_step_equals_unfused(n, rng):
    """Allgather(RandomK, ResidualMemory).step at world 1 through grace_randomk_step_w1 against the
    reference's four calls on the same engine: outputs and residuals bit-exact over 3 steps
    (duplicate indices included: they are drawn with replacement)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.randomk import RandomKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    gs = [np.random.default_rng(n + s).standard_normal(n).astype(np.float32) for s in range(3)]
    runs = []
    for fused in (True, False):
        comm = Allgather(RandomKCompressor(0.05, rng=rng), ResidualMemory(), 1)
        outs = []
        for s in range(3):
            g = torch.from_numpy(gs[s]).to("cuda")
            if fused:
                out = comm.step(g, "w")
            else:
                t = comm.memory.compensate(g, "w")
                payload, ctx = comm.compressor.compress(t, "w")
                comm.memory.update(t, "w", comm.compressor, payload, ctx)
                out = comm.send_receive(payload, "w", ctx)
            outs.append(out.cpu().numpy())
        runs.append((outs, comm.memory.residuals["w"].cpu().numpy()))
    (fo, fr), (uo, ur) = runs
    for s in range(3):
        assert same_bits(fo[s], uo[s]), s
    assert same_bits(fr, ur)
    assert np.count_nonzero(fo[-1]) > 0


@pytest.mark.parametrize("n,ratio", [((1 << 24) + 5, 0.01), (100003, 0.7), (8192, 0.3)])
def test_randomk_dense_step_equals_three_launch_step(n, ratio):
    """grace_randomk_step_w1_dense (indices grouped by chunk, one streaming pass) against
    grace_randomk_step_w1 (pass + gather + scatter): out and r' bit-identical, with many duplicate
    indices (ratio 0.7), special values and a partial last chunk."""
    from grace_amd import ops as G
    rng = np.random.default_rng(n)
    g0 = rng.standard_normal(n).astype(np.float32)
    g0[rng.choice(n, 3, replace=False)] = np.nan
    g0[rng.choice(n, 3, replace=False)] = -np.inf
    g0[rng.choice(n, 20, replace=False)] = -0.0
    r0 = (0.3 * rng.standard_normal(n)).astype(np.float32)
    k = G.ratio_k(n, ratio)
    idx = torch.from_numpy(rng.integers(0, n, k).astype(np.int64)).to("cuda")
    g = _t(g0)
    for has in (False, True):
        ra, rb = _t(r0), _t(r0)
        _, out_a = G.randomk_step_w1(g, ra, has, 1.0, 1.0, idx)
        out_b = G.randomk_step_w1_dense(g, rb, has, 1.0, 1.0, idx)
        assert same_bits(_np(out_b), _np(out_a)), has
        assert same_bits(_np(rb), _np(ra)), has
