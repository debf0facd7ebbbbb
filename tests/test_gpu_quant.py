"""GPU parity of the quantisation codecs (grace_amd/csrc/quant.hip) against the reference's golden
vectors.  Codewords are bit-exact given the reference's injected randomness and scale (norms / clamp
bound); scales computed on the device agree with the reference's CPU f32 reductions within 4 ulp."""
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


def test_qsgd_golden(golden):
    cases = golden.cases("quant", codec="qsgd")
    assert cases
    for c in cases:
        q, b = c.meta["quantum_num"], c.meta["bucket_size"]
        x = _t(c["x"].ravel())
        u = _t(c["u"])
        norms_ref = _t(c["norms"])
        # codewords with the reference's uniforms and norms: bit-exact
        codes, _ = ops.qsgd_compress(x, q, b, u=u, norms_in=norms_ref)
        assert same_bits(_np(codes), c["codes"].ravel()), c.name
        # norms computed on the device: within 4 ulp of torch's CPU f32 reduction
        codes2, norms = ops.qsgd_compress(x, q, b, u=u)
        assert ops.isclose_f32_ulps(_np(norms), c["norms"], 4), c.name
        agree = np.mean(_np(codes2).view(np.uint8 if q < 128 else np.uint16) ==
                        c["codes"].ravel().view(np.uint8 if q < 128 else np.uint16))
        assert agree > 0.999, (c.name, agree)
        # decompress with the reference payload: bit-exact
        dec = ops.qsgd_decompress(_t(c["codes"].ravel()), norms_ref, q, b, x.numel())
        assert same_bits(_np(dec), c["dec"].ravel()), c.name


def test_qsgd_compressor_torch_rng_matches_reference(golden):
    """rng='torch_cpu' consumes torch's global CPU generator exactly like the reference."""
    from grace_amd.dist.compressor.qsgd import QSGDCompressor
    for c in golden.cases("quant", codec="qsgd")[:6]:
        q, b = c.meta["quantum_num"], c.meta["bucket_size"]
        comp = QSGDCompressor(q, b, rng="torch_cpu")
        torch.manual_seed(c.meta["seed"])
        (codes, norms), shape = comp.compress(_t(c["x"]), "w")
        # norms may differ by ulps, so compare through the oracle given our norms
        exp, _ = O.qsgd_compress(c["x"], c["u"], q, b, norms=_np(norms))
        assert same_bits(_np(codes), exp), c.name


def test_terngrad_golden(golden):
    for c in golden.cases("quant", codec="terngrad"):
        x = c["x"].ravel()
        clip = np.array([O.terngrad_clip(x)], dtype=np.float32)
        codes, scal = ops.terngrad_compress(_t(x), clip=_t(clip), u=_t(c["u"]))
        assert np.array_equal(_np(codes), c["codes"].ravel()), c.name
        assert same_bits(_np(scal), c["scalar"].ravel()), c.name
        codes2, scal2 = ops.terngrad_compress(_t(x), u=_t(c["u"]))
        assert ops.isclose_f32_ulps(_np(scal2), c["scalar"].ravel(), 4), (c.name, _np(scal2), c["scalar"])
        dec = ops.terngrad_decompress(_t(c["codes"].ravel()), _t(c["scalar"].ravel()), x.size)
        assert same_bits(_np(dec), c["dec"].ravel()), c.name


def test_segmented_qsgd_and_terngrad_match_per_tensor():
    """One launch over many tensors == per-tensor launches (ResNet-style mixed shapes)."""
    rng = np.random.default_rng(0)
    sizes = [9408, 64, 64, 4096, 36864, 1, 129, 2048 * 10, 1000]
    xs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for n in sizes]
    flat = _t(np.concatenate(xs))
    u = rng.random(flat.numel(), dtype=np.float32)
    codes, norms = ops.qsgd_compress(flat, 127, 128, sizes=sizes, u=_t(u))
    tcodes, tscal = ops.terngrad_compress(flat, sizes=sizes, u=_t(u))
    off = 0
    noff = 0
    for i, (n, x) in enumerate(zip(sizes, xs)):
        c1, n1 = ops.qsgd_compress(_t(x), 127, 128, u=_t(u[off:off + n]))
        nb = -(-n // 128)
        assert same_bits(_np(codes[off:off + n]), _np(c1))
        assert same_bits(_np(norms[noff:noff + nb]), _np(n1))
        t1, s1 = ops.terngrad_compress(_t(x), u=_t(u[off:off + n]))
        assert same_bits(_np(tcodes[off:off + n]), _np(t1))
        assert same_bits(_np(tscal[i:i + 1]), _np(s1))
        off += n
        noff += nb
    dec = ops.qsgd_decompress(codes, norms, 127, 128, flat.numel(), sizes=sizes)
    exp = np.concatenate([O.qsgd_decode(*O.qsgd_compress(x, u[o:o + n], 127, 128, norms=None), 127, 128, n)
                          for x, n, o in zip(xs, sizes, np.cumsum([0] + sizes[:-1]))])
    assert np.allclose(_np(dec), exp, rtol=1e-5, atol=1e-7)


def test_world2_qsgd_terngrad_aggregate(golden):
    r0, r1 = golden.case("world2", "rank0"), golden.case("world2", "rank1")
    codes = _t(np.concatenate([r0["qsgd_codes"], r1["qsgd_codes"]]))
    norms = _t(np.concatenate([r0["qsgd_norms"], r1["qsgd_norms"]]))
    out = ops.qsgd_decompress(codes, norms, 127, 128, 4099, world=2, aggregate=True, divisor=2.0)
    assert same_bits(_np(out), r0["qsgd_out"].ravel())
    codes = _t(np.concatenate([r0["tern_codes"], r1["tern_codes"]]))
    scal = _t(np.concatenate([r0["tern_scalar"], r1["tern_scalar"]]))
    out = ops.terngrad_decompress(codes, scal, 4099, world=2, aggregate=True, divisor=2.0)
    assert same_bits(_np(out), r0["tern_out"].ravel())


def test_qsgd_device_rng_properties():
    x = np.random.default_rng(1).standard_normal(1 << 20).astype(np.float32) * 0.01
    codes, norms = ops.qsgd_compress(_t(x), 127, 128, seed=1234)
    norms_np = _np(norms)
    level = (np.float32(1) / np.repeat(norms_np, 128)[: x.size] * np.float32(127)) * np.abs(x)
    c = np.abs(_np(codes).astype(np.int32))
    assert np.all((c == np.floor(level)) | (c == np.floor(level) + 1))
    # unbiased: mean of the decode matches x in aggregate
    dec = _np(ops.qsgd_decompress(codes, norms, 127, 128, x.size))
    assert abs(float(np.mean(dec - x))) < 1e-5
    # deterministic for a given seed
    codes2, _ = ops.qsgd_compress(_t(x), 127, 128, seed=1234)
    assert torch.equal(codes, codes2)


@pytest.mark.parametrize("q,variant", [(127, 0), (255, 0), (127, 1)])
def test_qsgd_device_rng_fast_path_bit_exact(q, variant):
    """The device-generator encoder (qsgd_encode128_pipe_kernel: pipelined, partial / unaligned
    buckets encoded afterwards) against the injected-stream encoder fed the same uniforms
    (tests/device_rng.py), and against the oracle; the fused world-1 step against its decode.
    Segments: whole buckets, a partial last bucket, unaligned starts, a 2-element segment."""
    from tests.device_rng import qsgd_bucket128_uniforms
    rng = np.random.default_rng(11 + q + variant)
    sizes = [128 * 300, 1001, 4099, 2, 128 * 37, 64, 3, 128 * 21 + 5, 7777]
    flat = (rng.standard_normal(sum(sizes)) * 0.01).astype(np.float32)
    if variant == 1:
        flat[[5, 40000, 45000]] = [np.inf, np.nan, -np.inf]
    seed = 0xC0FFEE + q
    u = qsgd_bucket128_uniforms(seed, sizes)
    codes, norms = ops.qsgd_compress(_t(flat), q, 128, sizes=sizes, variant=variant, seed=seed)
    codes_u, norms_u = ops.qsgd_compress(_t(flat), q, 128, sizes=sizes, variant=variant, u=_t(u))
    assert same_bits(_np(norms), _np(norms_u))
    assert same_bits(_np(codes), _np(codes_u))
    if variant == 0:
        off, noff = 0, 0
        norms_np = _np(norms)
        for n in sizes:
            nb = (n + 127) // 128
            exp_c, _ = O.qsgd_compress(flat[off:off + n], u[off:off + n], q, 128, norms=norms_np[noff:noff + nb])
            assert same_bits(_np(codes)[off:off + n], exp_c), (n, off)
            off, noff = off + n, noff + nb
    dec = ops.qsgd_decompress(codes, norms, q, 128, flat.size, sizes=sizes, variant=variant)
    fused = ops.qsgd_step_w1(_t(flat), q, sizes=sizes, variant=variant, seed=seed)
    assert same_bits(_np(fused), _np(dec))


def test_natural_vs_oracle():
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.standard_normal(100000).astype(np.float32) * 3,
                        np.array([0, -0.0, np.inf, -np.inf, np.nan, 1e-45, 2 ** -110, 2.0 ** 20], dtype=np.float32)])
    ri = rng.integers(0, 0x7FFFFF, x.size, dtype=np.int32)
    codes = ops.natural_compress(_t(x), rand_int=_t(ri))
    exp = O.natural_compress(x, ri)
    assert np.array_equal(_np(codes), exp)
    assert same_bits(_np(ops.natural_decompress(codes, x.size, 0)), O.natural_decode(exp))


def test_cnat_vs_oracle():
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.standard_normal(100000).astype(np.float32),
                        np.array([1.0, 0.75, -1.0, 0.0, 2.0 ** -109, 2.0 ** -110, 2.0 ** 20, -(2.0 ** -120)],
                                 dtype=np.float32)])
    codes = ops.cnat_compress(_t(x), deterministic=True)
    exp = O.cnat_compress(x)
    assert np.array_equal(_np(codes), exp)
    r = rng.random(x.size, dtype=np.float32)
    codes = ops.cnat_compress(_t(x), rand=_t(r))
    exp = O.cnat_compress(x, r)
    assert np.array_equal(_np(codes), exp)
    assert same_bits(_np(ops.natural_decompress(codes, x.size, 1)), O.cnat_decode(exp))


def test_fp16_golden(golden):
    from grace_amd.dist.compressor.fp16 import FP16Compressor
    comp = FP16Compressor()
    for c in golden.cases("quant", codec="fp16"):
        (h,), ctx = comp.compress(_t(c["x"]), "w")
        assert same_bits(_np(h), c["half"]), c.name
        assert same_bits(_np(comp.decompress([h], ctx)), c["dec"]), c.name


@pytest.mark.parametrize("cls", ["qsgd", "terngrad", "natural", "natural_cuda"])
def test_allgather_world1_step(cls):
    """Communicator.step through each quantiser at world 1 = (0 + decompress(compress(x))) / 1."""
    from grace_amd.dist.helper import grace_from_params
    comm = grace_from_params({"compressor": cls, "memory": "none", "communicator": "allgather", "world_size": 1})
    x = _t(np.random.default_rng(4).standard_normal(5000).astype(np.float32) * 0.01)
    torch.manual_seed(0)
    out = comm.step(x, "w")
    assert out.shape == x.shape and torch.isfinite(out).all()
    # stochastic codecs are unbiased: the mean error is small against the spread of x
    bias = abs(float((out - x).mean()))
    assert bias < 0.1 * float(x.std())


@pytest.mark.parametrize("q,bucket", [(127, 8), (127, 100), (127, 128), (255, 128), (127, 256), (200, 37)])
def test_segmented_qsgd_bucket_and_code_variants(q, bucket):
    """Segmented encode/decode at odd bucket sizes, fp16 codewords (q >= 128) and ragged segment
    offsets (exercises the 16-element decode fast path, its bucket split and the slow path)."""
    rng = np.random.default_rng(5)
    sizes = [37, 1, 4099, 16, 15, 128 * 7 + 3, 2048, 1000]
    xs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for n in sizes]
    flat = np.concatenate(xs)
    u = rng.random(flat.size, dtype=np.float32)
    codes, norms = ops.qsgd_compress(_t(flat), q, bucket, sizes=sizes, u=_t(u))
    dec = _np(ops.qsgd_decompress(codes, norms, q, bucket, flat.size, sizes=sizes))
    norms_np = _np(norms)
    off = noff = 0
    for n, x in zip(sizes, xs):
        nb = -(-n // bucket)
        exp_c, _ = O.qsgd_compress(x, u[off:off + n], q, bucket, norms=norms_np[noff:noff + nb])
        assert same_bits(_np(codes[off:off + n]), exp_c), (n, q, bucket)
        exp_d = O.qsgd_decode(exp_c, norms_np[noff:noff + nb], q, bucket, n)
        assert same_bits(dec[off:off + n], exp_d), (n, q, bucket)
        off += n
        noff += nb


def test_segmented_terngrad_decode_world3_ragged():
    """W = 3 aggregate over ragged segments with a code stride that is not 16-B aligned."""
    rng = np.random.default_rng(6)
    sizes = [5, 33, 4096 + 7, 1, 300]
    n = sum(sizes)
    codes = rng.integers(-1, 2, size=3 * n, dtype=np.int8)
    scal = rng.random(3 * len(sizes), dtype=np.float32)
    out = _np(ops.terngrad_decompress(_t(codes), _t(scal), n, sizes=sizes, world=3, aggregate=True, divisor=3.0))
    seg = np.repeat(np.arange(len(sizes)), sizes)
    decs = [codes[w * n:(w + 1) * n].astype(np.float32) * scal[w * len(sizes) + seg] for w in range(3)]
    exp = (O.python_sum(decs) / np.float32(3)).astype(np.float32)
    assert same_bits(out, exp)


def test_qsgd_cuda_variant_vs_oracle_with_specials():
    """QSGDCompressor_CUDA semantics (variant 1) on the bucket-of-128 row kernels: f64 norms over
    finite elements, NaN/Inf -> -128, decoded back to NaN; ragged segments (parity unpinned: the
    oracle restates qsgd_cuda.cu:320-388, CUDA-only in the reference)."""
    rng = np.random.default_rng(8)
    sizes = [130, 1, 4096, 257, 128]
    xs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for n in sizes]
    xs[0][[3, 77]] = [np.nan, np.inf]
    xs[2][1000:1128] = 0.0                       # an all-zero bucket
    xs[3][-1] = -np.inf
    flat = np.concatenate(xs)
    u = rng.random(flat.size, dtype=np.float32)
    codes, norms = ops.qsgd_compress(_t(flat), 127, 128, sizes=sizes, variant=1, u=_t(u))
    dec = _np(ops.qsgd_decompress(codes, norms, 127, 128, flat.size, sizes=sizes, variant=1))
    off = noff = 0
    cn, nn = _np(codes), _np(norms)
    for n, x in zip(sizes, xs):
        nb = -(-n // 128)
        _, ref_n = O.qsgd_cuda_compress(x, u[off:off + n], 127, 128)
        # device norms: f64 sums in another order, so within 1 ulp of the oracle's; the codewords
        # are then checked bit-exactly given the device norms
        assert ops.isclose_f32_ulps(nn[noff:noff + nb], ref_n.astype(np.float32), 1), n
        exp_c, exp_n = O.qsgd_cuda_compress(x, u[off:off + n], 127, 128, norms=nn[noff:noff + nb])
        assert np.array_equal(cn[off:off + n], exp_c), n
        d = dec[off:off + n]
        assert np.all(np.isnan(d[exp_c == -128]))
        ok = exp_c != -128
        exp_d = ((exp_n.astype(np.float32)[np.arange(n) // 128] / np.float32(127)).astype(np.float32)
                 * exp_c.astype(np.float32)).astype(np.float32)
        assert same_bits(d[ok], exp_d[ok]), n
        off += n
        noff += nb


@pytest.mark.parametrize("world", [2, 5])
def test_qsgd_bucket_decoder_multi_rank_aggregate(world):
    """The bucket-of-128 decoder's rank-ordered W-payload aggregate and divisor against the oracle
    over ragged segments (including a code stride that is not a multiple of 4)."""
    rng = np.random.default_rng(world)
    sizes = [5, 300, 4096, 1, 131]
    n = sum(sizes)
    nb = sum(-(-s // 128) for s in sizes)
    cs, ns = [], []
    for w in range(world):
        x = (rng.standard_normal(n) * 0.01).astype(np.float32)
        c, nm = ops.qsgd_compress(_t(x), 127, 128, sizes=sizes, u=_t(rng.random(n, dtype=np.float32)))
        cs.append(_np(c))
        ns.append(_np(nm))
    out = _np(ops.qsgd_decompress(_t(np.concatenate(cs)), _t(np.concatenate(ns)), 127, 128, n, sizes=sizes,
                                  world=world, aggregate=True, divisor=float(world)))
    bidx = np.concatenate([sum(-(-sizes[j] // 128) for j in range(i)) + np.arange(s) // 128
                           for i, s in enumerate(sizes)])
    decs = [((ns[w][bidx] / np.float32(127)).astype(np.float32) * cs[w].astype(np.float32)).astype(np.float32)
            for w in range(world)]
    exp = (O.python_sum(decs) / np.float32(world)).astype(np.float32)
    assert nb == ns[0].size
    assert same_bits(out, exp)


def test_terngrad_nan_clamp_bound_propagates():
    """terngrad.py:13-16: torch.clamp with a NaN bound gives NaN everywhere, so the scalar is NaN and
    every code 0.  The bound is NaN when the clip is injected as NaN or when the tensor holds an inf
    (std = NaN).  Ragged segments around an inf segment, oracle bit-exact (scalars and codes)."""
    rng = np.random.default_rng(21)
    sizes = [5, 4099, 13, 70001, 7]
    xs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for n in sizes]
    xs[1][17] = np.inf
    xs[3][0] = -np.inf
    flat = np.concatenate(xs)
    u = rng.random(flat.size, dtype=np.float32)
    offs = np.cumsum([0] + sizes[:-1])
    clips = np.array([O.terngrad_clip(x) for x in xs], dtype=np.float32)
    assert np.isnan(clips[1]) and np.isnan(clips[3]) and not np.isnan(clips[0])
    for clip in (None, clips):
        codes, scal = ops.terngrad_compress(_t(flat), sizes=sizes, u=_t(u), clip=None if clip is None else _t(clip))
        exp = [O.terngrad_compress(x, u[o:o + n], clip=None if clip is None else clip[i])
               for i, (x, n, o) in enumerate(zip(xs, sizes, offs))]
        exp_s = np.concatenate([e[1] for e in exp])
        s = _np(scal)
        assert np.isnan(s[1]) and np.isnan(s[3])
        if clip is None:   # device statistics: NaN where the oracle is NaN, else within 4 ulp
            fin = ~np.isnan(exp_s)
            assert same_bits(s[~fin], exp_s[~fin]) and ops.isclose_f32_ulps(s[fin], exp_s[fin], 4)
        else:
            assert same_bits(s, exp_s)
            assert np.array_equal(_np(codes), np.concatenate([e[0] for e in exp]))
        c = _np(codes)
        assert not c[offs[1]:offs[1] + sizes[1]].any() and not c[offs[3]:offs[3] + sizes[3]].any()


def test_terngrad_workspace_many_units_alternating():
    """A call with hundreds of units alternating with 3-unit calls on the same workspace: each
    segment's arrival counter must not share memory with a smaller call's partials (the
    struct-of-arrays layout sized by nunits put them there once a segment started past unit 64)."""
    rng = np.random.default_rng(11)
    sizes = [16384 * 2 + 7] * 120
    flat = (rng.standard_normal(sum(sizes)) * 0.01).astype(np.float32)
    u = rng.random(flat.size, dtype=np.float32)
    for _ in range(2):
        codes, scal = ops.terngrad_compress(_t(flat), sizes=sizes, u=_t(u))
        off = 0
        for i, s in enumerate(sizes):
            c1, s1 = ops.terngrad_compress(_t(flat[off:off + s]), u=_t(u[off:off + s]))
            assert same_bits(_np(codes[off:off + s]), _np(c1)), i
            assert same_bits(_np(scal[i:i + 1]), _np(s1)), i
            off += s


def test_terngrad_workspace_reuse_across_shapes():
    """The TernGrad workspace is shared by calls of different unit counts: its arrival counters
    must stay zeroed whichever shape ran before (a regression the segmented test first caught).
    Segmented results must equal each tensor compressed on its own, call after call."""
    rng = np.random.default_rng(9)
    shapes = [[70000, 3], [5], [16384 * 3 + 1, 2, 40000], [9]]
    for sizes in shapes * 2:
        xs = [(rng.standard_normal(s) * 0.01).astype(np.float32) for s in sizes]
        flat = np.concatenate(xs)
        u = rng.random(flat.size, dtype=np.float32)
        codes, scal = ops.terngrad_compress(_t(flat), sizes=sizes, u=_t(u))
        off = 0
        for i, (s, x) in enumerate(zip(sizes, xs)):
            c1, s1 = ops.terngrad_compress(_t(x), u=_t(u[off:off + s]))
            assert same_bits(_np(codes[off:off + s]), _np(c1)), (sizes, i)
            assert same_bits(_np(scal[i:i + 1]), _np(s1)), (sizes, i)
            off += s


@pytest.mark.parametrize("n,off", [(1, 0), (5, 1), (4099, 0), (4099, 3), (1 << 20, 1)])
def test_byte_codecs_vectorised_edges(n, off):
    """natural / cnat / fp16 quad kernels: ragged tails and unaligned views (offset slices)."""
    rng = np.random.default_rng(n + off)
    base = rng.standard_normal(n + off).astype(np.float32) * 3
    x = base[off:]
    xd = _t(base)[off:]
    ri = rng.integers(0, 0x7FFFFF, n + off, dtype=np.int32)
    rd = _t(ri)[off:]
    codes = ops.natural_compress(xd, rand_int=rd)
    assert np.array_equal(_np(codes), O.natural_compress(x, ri[off:]))
    assert same_bits(_np(ops.natural_decompress(codes, n, 0)), O.natural_decode(O.natural_compress(x, ri[off:])))
    u = rng.random(n + off, dtype=np.float32)
    cc = ops.cnat_compress(xd, rand=_t(u)[off:])
    assert np.array_equal(_np(cc), O.cnat_compress(x, u[off:]))
    assert same_bits(_np(ops.natural_decompress(cc, n, 1)), O.cnat_decode(O.cnat_compress(x, u[off:])))
    h = ops.fp16_compress(xd)
    assert np.array_equal(_np(h).view(np.uint16), O.fp16_compress(x).view(np.uint16))
    assert same_bits(_np(ops.fp16_decompress(h)), O.fp16_decode(O.fp16_compress(x)))


@pytest.mark.parametrize("world,average", [(1, True), (2, True), (3, False)])
def test_fp16_allgather_fused_decode(world, average):
    """FP16Compressor.decode_aggregate_gathered (grace_fp16_decompress_aggregate): the W gathered
    f16 payloads decoded, summed from 0 in rank order and divided by W when averaging, in one pass
    -- bit-exact against Python's sum of the per-rank decodes (allgather.py:40-45), including -0,
    inf/NaN and an odd length (scalar tail)."""
    from grace_amd.dist.compressor.fp16 import FP16Compressor
    rng = np.random.default_rng(world)
    n = 100003
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
    xs[0][:4] = [-0.0, np.inf, np.nan, 7e4]
    hs = [O.fp16_compress(x) for x in xs]
    comp = FP16Compressor()
    comp.average = average
    gathered = [_t(np.concatenate(hs))]
    out = _np(comp.decode_aggregate_gathered(gathered, (torch.float32, torch.Size([n])), world))
    exp = np.float32(0.0) + O.fp16_decode(hs[0])
    for h in hs[1:]:
        exp = (exp + O.fp16_decode(h)).astype(np.float32)
    if average:
        exp = (exp / np.float32(world)).astype(np.float32)
    assert same_bits(out, exp)


def test_fp16_allgather_step_world1():
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.fp16 import FP16Compressor
    from grace_amd.dist.memory.none import NoneMemory
    x = np.random.default_rng(9).standard_normal((33, 65)).astype(np.float32)
    out = _np(Allgather(FP16Compressor(), NoneMemory(), 1).step(_t(x), "w"))
    assert out.shape == x.shape
    assert same_bits(out.ravel(), np.float32(0.0) + O.fp16_decode(O.fp16_compress(x.ravel())))


@pytest.mark.parametrize("cls,rng", [("natural", "device"), ("cnat", "device"), ("cnat", "deterministic"),
                                     ("fp16", None)])
@pytest.mark.parametrize("n", [1, 7, 4096, 1000003])
def test_cast_world1_fused_step_equals_unfused(cls, rng, n):
    """grace_cast_step_w1 (one pass, codes never stored) == compress -> Allgather decode at world 1
    -> (0 + d) / 1 through the separate kernels, bit for bit, on the same device generator draws
    (two compressors stepped in lockstep: the fused one and one whose fused path is disabled)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.fp16 import FP16Compressor
    from grace_amd.dist.compressor.natural import NaturalCompressor, NaturalCompressor_CUDA
    from grace_amd.dist.memory.none import NoneMemory
    mk = {"natural": lambda: NaturalCompressor(rng=rng), "cnat": lambda: NaturalCompressor_CUDA(rng=rng),
          "fp16": FP16Compressor}[cls]
    fused, plain = mk(), mk()
    plain.fused_step = lambda *a: None
    cf, cp = Allgather(fused, NoneMemory(), 1), Allgather(plain, NoneMemory(), 1)
    x = np.random.default_rng(n).standard_normal(n).astype(np.float32)
    x[: min(n, 3)] = [-0.0, 3e-39, -7e4][: min(n, 3)]
    xd = _t(x)
    for step in range(2):
        a, b = _np(cf.step(xd, "w")), _np(cp.step(xd, "w"))
        assert same_bits(a, b), (cls, rng, n, step)


@pytest.mark.parametrize("cls,q", [("qsgd", 127), ("qsgd", 255), ("qsgd_cuda", 127)])
def test_qsgd_world1_fused_step_equals_unfused(cls, q):
    """grace_qsgd_step_w1 == compress -> Allgather decode at world 1, bit for bit (same device
    generator draws, and the injected torch_cpu stream), on a tensor with a ragged last bucket and
    NaN / Inf / zero buckets; plus the segmented ResNet-50 set through ops.qsgd_step_w1."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.qsgd import QSGDCompressor, QSGDCompressor_CUDA
    from grace_amd.dist.memory.none import NoneMemory
    mk = QSGDCompressor if cls == "qsgd" else QSGDCompressor_CUDA
    x = (np.random.default_rng(q).standard_normal(100003) * 0.01).astype(np.float32)
    x[128:256] = 0.0
    x[300] = np.inf
    x[700] = np.nan
    for rng in ("device", "torch_cpu"):
        fused, plain = mk(q, 128, rng=rng), mk(q, 128, rng=rng)
        plain.fused_step = lambda *a: None
        cf, cp = Allgather(fused, NoneMemory(), 1), Allgather(plain, NoneMemory(), 1)
        for step in range(2):
            torch.manual_seed(step)
            a = _np(cf.step(_t(x), "w"))
            torch.manual_seed(step)
            b = _np(cp.step(_t(x), "w"))
            assert same_bits(a, b), (cls, q, rng, step)
    from bench import resnet50_shapes
    sizes = [int(np.prod(s)) for s in resnet50_shapes()]
    flat = _t((np.random.default_rng(1).standard_normal(sum(sizes)) * 0.01).astype(np.float32))
    variant = 0 if cls == "qsgd" else 1
    codes, norms = ops.qsgd_compress(flat, q, 128, sizes=sizes, variant=variant, seed=7)
    dec = ops.qsgd_decompress(codes, norms, q, 128, flat.numel(), sizes=sizes, variant=variant, aggregate=True)
    assert same_bits(_np(ops.qsgd_step_w1(flat, q, sizes=sizes, variant=variant, seed=7)), _np(dec))


def test_terngrad_world1_fused_step_equals_unfused():
    """grace_terngrad_step_w1 == compress -> Allgather decode at world 1, bit for bit (device draws
    and the injected torch_cpu stream, int8 and 2-bit wires), ragged tail and a zero tensor; plus the
    segmented ResNet-50 set through ops.terngrad_step_w1 against terngrad_compress/decompress."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.terngrad import TernGradCompressor
    from grace_amd.dist.memory.none import NoneMemory
    x = (np.random.default_rng(5).standard_normal(100003) * 0.01).astype(np.float32)
    for xin in (x, np.zeros(4099, np.float32)):
        for rng in ("device", "torch_cpu"):
            for wire in ("int8", "2bit"):
                fused, plain = TernGradCompressor(rng=rng, wire=wire), TernGradCompressor(rng=rng, wire=wire)
                plain.fused_step = lambda *a: None
                cf, cp = Allgather(fused, NoneMemory(), 1), Allgather(plain, NoneMemory(), 1)
                for step in range(2):
                    torch.manual_seed(step)
                    a = _np(cf.step(_t(xin), "w"))
                    torch.manual_seed(step)
                    b = _np(cp.step(_t(xin), "w"))
                    assert same_bits(a, b), (rng, wire, step, xin.size)
    from bench import resnet50_shapes
    sizes = [int(np.prod(s)) for s in resnet50_shapes()]
    flat = _t((np.random.default_rng(2).standard_normal(sum(sizes)) * 0.01).astype(np.float32))
    codes, scal = ops.terngrad_compress(flat, sizes=sizes, seed=9)
    dec = ops.terngrad_decompress(codes, scal, flat.numel(), sizes=sizes, aggregate=True)
    assert same_bits(_np(ops.terngrad_step_w1(flat, sizes=sizes, seed=9)), _np(dec))
