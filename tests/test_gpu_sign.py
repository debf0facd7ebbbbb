"""GPU parity of the sign-family HIP kernels against the reference's golden vectors."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
ROWS_COLS = (4099, 1)
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def test_signsgd_golden(golden):
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    comp = SignSGDCompressor()
    for c in golden.cases("sign", codec="signsgd"):
        if "codes" not in c:
            continue
        (codes,), shape = comp.compress(_t(c["x"]), "w")
        assert np.array_equal(_np(codes), c["codes"].ravel()), c.name
        dec = comp.decompress([codes], shape)
        assert same_bits(_np(dec), c["dec"]), c.name
        decs = [comp.decompress(comp.compress(_t(c[f"agg_in{i}"]), "w")[0], shape) for i in range(3)]
        assert same_bits(_np(comp.aggregate(decs)), c["agg"]), c.name


def test_signsgd_step_world1(golden):
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    c = golden.case("sign", "signsgd_step_w1")
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
    assert same_bits(_np(comm.step(_t(c["x"]), "w")), c["out"])
    # the generic path gives the same
    payload, ctx = comm.compressor.compress(_t(c["x"]), "w")
    assert same_bits(_np(comm.send_receive(payload, "w", ctx)), c["out"])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sign_majority_matches_oracle(world):
    from grace_amd import ops
    n = 4099 * 4
    xs = [np.random.default_rng(w).standard_normal(n).astype(np.float32) for w in range(world)]
    codes = torch.cat([ops.sign_encode(_t(x)) for x in xs])
    out = ops.sign_majority(codes, world, n)
    exp = O.sign_aggregate([O.sign_decode(O.sign_encode(x)) for x in xs])
    assert same_bits(_np(out), exp)


def test_signum_golden(golden):
    from grace_amd.dist.compressor.signum import SignumCompressor
    c = golden.case("sign", "signum_seq")
    comp = SignumCompressor(0.9)
    for s in range(3):
        (codes,), shape = comp.compress(_t(c[f"x{s}"]), "w")
        assert np.array_equal(_np(codes), c[f"codes{s}"]), s
        assert same_bits(_np(comp.momentums["w"]), c[f"mom{s}"].ravel()), s
        assert same_bits(_np(comp.decompress([codes], shape)), c[f"dec{s}"]), s


def test_efsignsgd_golden(golden):
    """Codewords bit-exact; the |x| mean within 2 ulp (f64 device reduction vs torch's f32
    cascade); decode bit-exact given the same mean."""
    from grace_amd.dist.compressor.efsignsgd import EFSignSGDCompressor
    from grace_amd.dist.memory.efsignsgd import EFSignSGDMemory
    from grace_amd.ops import isclose_f32_ulps
    c = golden.case("sign", "efsignsgd_seq")
    comp, mem = EFSignSGDCompressor(0.1), EFSignSGDMemory(0.1)
    for s in range(3):
        # feed the reference's residual so each step is checked independently
        if s > 0:
            mem.residuals["w"] = _t(c[f"res{s - 1}"])
        t = mem.compensate(_t(c[f"x{s}"]), "w")
        assert same_bits(_np(t), c[f"t{s}"]), s
        (mean, codes), shape = comp.compress(t, "w")
        assert np.array_equal(_np(codes), c[f"codes{s}"]), s
        assert isclose_f32_ulps(_np(mean), c[f"mean{s}"], 2), (s, _np(mean), c[f"mean{s}"])
        dec = comp.decompress((_t(c[f"mean{s}"]), codes), shape)
        assert same_bits(_np(dec), c[f"dec{s}"]), s


def test_onebit_golden(golden):
    from grace_amd.dist.compressor.onebit import OneBitCompressor
    from grace_amd.ops import isclose_f32_ulps
    for c in golden.cases("sign", codec="onebit"):
        for quirk, key in ((True, "dec_quirk"), (False, "dec_fixed")):
            comp = OneBitCompressor(compat_uint8_not=quirk)
            (mask0, m0, m1), shape = comp.compress(_t(c["x"]), "w")
            assert np.array_equal(_np(mask0), c["mask0"]), c.name
            assert isclose_f32_ulps(_np(m0), c["mean0"], 4), (c.name, _np(m0), c["mean0"])
            assert isclose_f32_ulps(_np(m1), c["mean1"], 4), (c.name, _np(m1), c["mean1"])
            dec = comp.decompress((mask0, _t(c["mean0"]), _t(c["mean1"])), shape)
            assert same_bits(_np(dec), c[key]), (c.name, quirk)


def test_no_cpu_path():
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.ops import GraceDeviceError
    with pytest.raises(GraceDeviceError):
        SignSGDCompressor().compress(torch.zeros(8), "w")


def test_w1_step_output_reuse_never_clobbers_a_held_result():
    """The W=1 fused sign step reuses its output buffer only when the caller dropped the previous
    result (ops.reusable_output); results the caller keeps stay intact."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
    rng = np.random.default_rng(9)
    xs = [rng.standard_normal(4099).astype(np.float32) for _ in range(4)]
    kept = [comm.step(_t(x), "w") for x in xs]                  # all held: four distinct buffers
    assert len({k.data_ptr() for k in kept}) == 4
    for k, x in zip(kept, xs):
        assert np.array_equal(_np(k), np.where(x >= 0, 1.0, -1.0).astype(np.float32))
    p1 = comm.step(_t(xs[0]), "w").data_ptr()                    # dropped at once -> reused
    p2 = comm.step(_t(xs[1]), "w").data_ptr()
    assert p1 == p2
    out = comm.step(_t(xs[2]).view(ROWS_COLS), "w")             # 2-D input keeps its shape
    assert out.shape == ROWS_COLS


def test_w1_step_output_reuse_respects_views():
    """A caller that keeps only a view / reshape / slice of the result (``grads.append(step(g).view(-1))``)
    or gets a view back (non-contiguous input) must never see that result overwritten by a later
    step: the reuse guard checks the storage's use count, not just the object's."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
    rng = np.random.default_rng(10)
    xs = [rng.standard_normal(4099).astype(np.float32) for _ in range(6)]
    exp = [np.where(x >= 0, 1.0, -1.0).astype(np.float32) for x in xs]
    held = [comm.step(_t(x), "w").view(-1) for x in xs[:2]]        # views only
    held.append(comm.step(_t(xs[2]), "w")[1:])                     # a slice only
    held.append(comm.step(_t(xs[3]), "w").reshape(1, -1))          # a reshape (view) only
    for h, e, cut in zip(held, exp, (0, 0, 1, 0)):
        assert np.array_equal(_np(h).ravel(), e[cut:])
    # non-contiguous input: the result the caller gets is a view of the cached output
    m = rng.standard_normal((64, 96)).astype(np.float32)
    nc = _t(m).t()
    assert not nc.is_contiguous()
    a = comm.step(nc, "w")
    b = comm.step(_t(-m).t(), "w")
    assert np.array_equal(_np(a), np.where(m.T >= 0, 1.0, -1.0).astype(np.float32))
    assert np.array_equal(_np(b), np.where(-m.T >= 0, 1.0, -1.0).astype(np.float32))
    for h, e, cut in zip(held, exp, (0, 0, 1, 0)):                # still intact after more steps
        assert np.array_equal(_np(h).ravel(), e[cut:])


def _planted(n, seed):
    """f32[n] standard normal with +-0, NaN, +-inf and denormals planted at both ends and inside."""
    x = np.random.default_rng(seed).standard_normal(n).astype(np.float32)
    specials = np.array([0.0, -0.0, np.nan, -np.nan, np.inf, -np.inf, 1e-45, -1e-45], dtype=np.float32)
    for base in (0, n // 3, n // 2 + 1, n - len(specials)):
        x[base:base + len(specials)] = specials
    return x


@pytest.mark.parametrize("shape", [(1 << 20,), ((1 << 20) + 3,), (1024, 1024)],
                         ids=["n=2^20", "n=2^20+3", "1024x1024"])
def test_signsgd_configs0_at_size(shape):
    """BASELINE configs[0] at its own size: Allgather(SignSGD, NoneMemory, 1).step on one 4 MiB f32
    tensor (n = 1,048,576; plus a ragged n and a 2-D view), bit-exact against the oracle's
    sign_aggregate([sign_decode(sign_encode(x))]) with +-0 / NaN / +-inf / denormals planted; the
    unfused compress -> decompress -> aggregate at the same size gives the same bits
    (grace_dl/dist/compressor/signsgd.py:6-30)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = int(np.prod(shape))
    x = _planted(n, 40 + n % 7)
    exp = O.sign_aggregate([O.sign_decode(O.sign_encode(x))]).reshape(shape)
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
    xt = _t(x).view(shape)
    for _ in range(2):                        # the second step reuses the dropped output buffer
        out = comm.step(xt, "w")
        assert out.shape == torch.Size(shape)
        assert same_bits(_np(out), exp)
    comp = comm.compressor
    (codes,), ctx = comp.compress(xt, "w")
    assert np.array_equal(_np(codes), O.sign_encode(x))
    dec = comp.decompress([codes], ctx)
    assert same_bits(_np(dec), O.sign_decode(O.sign_encode(x)).reshape(shape))
    assert same_bits(_np(comp.aggregate([dec])), exp)
    assert same_bits(_np(comm.send_receive([codes], "w", ctx)), exp)
    # x itself is never written
    assert same_bits(_np(xt).ravel(), x)
