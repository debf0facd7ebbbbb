"""Packed wire formats (grace_amd/csrc/wire.hip): 1-bit sign codes and the 2-bit layout of
grace_dl/tensorflow/compressor/packing.py (oracle restatement; TensorFlow is absent, so the
2-bit layout is parity-unpinned against the reference's own run)."""
import numpy as np
import pytest
import torch

from grace_amd import ops
from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, (1 << 20) + 5])
def test_pack_bits_roundtrip(n):
    codes = np.random.default_rng(n).integers(0, 2, n).astype(np.uint8)
    words = ops.pack_bits(_t(codes))
    exp = np.packbits(codes, bitorder="little")
    got = _np(words).view(np.uint8)[:exp.size]
    assert np.array_equal(got, exp)
    assert np.array_equal(_np(ops.unpack_bits(words, n)), codes)


@pytest.mark.parametrize("n", [1, 31, 32, 33, 255, 256, 1023, 4097, (1 << 20) + 5])
@pytest.mark.parametrize("offset", [0, 1])
def test_sign_encode_bits_equals_pack_of_codes(n, offset):
    """grace_sign_encode_bits (one pass) == pack_bits(sign_encode(x)), incl. -0, NaN, +-inf, ragged
    tails and a misaligned input view (offset 1: the scalar path)."""
    rng = np.random.default_rng(n + offset)
    x = rng.standard_normal(n + offset).astype(np.float32)
    for v in (-0.0, 0.0, np.nan, np.inf, -np.inf):
        x[rng.integers(0, n + offset, 3)] = v
    xt = _t(x)[offset:]
    got = _np(ops.sign_encode_bits(xt))
    exp = _np(ops.pack_bits(ops.sign_encode(xt)))
    assert np.array_equal(got, exp)
    assert np.array_equal(got.view(np.uint8)[:(n + 7) // 8],
                          np.packbits(O.sign_encode(x[offset:]).astype(np.uint8), bitorder="little"))


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8, 16])
def test_majority_bits_equals_u8(world):
    n = 100003
    rng = np.random.default_rng(world)
    codes = [rng.integers(0, 2, n).astype(np.uint8) for _ in range(world)]
    u8 = _np(ops.sign_majority(_t(np.concatenate(codes)), world, n))
    words = torch.cat([ops.pack_bits(_t(c)) for c in codes])
    bits = _np(ops.sign_majority_bits(words, world, n))
    assert same_bits(bits, u8)
    assert same_bits(u8, O.sign_aggregate([O.sign_decode(c) for c in codes]))


@pytest.mark.parametrize("n", [1, 3, 4, 5, 8, 4099, 1 << 16])
def test_pack2_matches_packing_py(n):
    vals = np.random.default_rng(n).integers(0, 4, n).astype(np.uint8)
    enc = _np(ops.pack2(_t(vals)))
    assert np.array_equal(enc, O.pack2_encode(vals))
    assert np.array_equal(_np(ops.unpack2(_t(enc), n)), O.pack2_decode(enc, n).astype(np.uint8))
    codes = (vals % 3).astype(np.int8) - 1
    packed = ops.tern_pack(_t(codes))
    assert np.array_equal(_np(packed), O.pack2_encode(codes.astype(np.int64) + 1))
    assert np.array_equal(_np(ops.tern_unpack(packed, n)), codes)


def test_packed_compressors_equal_default_wire():
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.compressor.terngrad import TernGradCompressor
    x = _t(np.random.default_rng(0).standard_normal(50001).astype(np.float32))
    a, b = SignSGDCompressor(), SignSGDCompressor(wire="bits")
    pa, ctx = a.compress(x, "w")
    pb, _ = b.compress(x, "w")
    assert pb[0].numel() * 4 * 8 >= x.numel() and pb[0].numel() * 4 < pa[0].numel() // 7
    assert same_bits(_np(a.decompress(pa, ctx)), _np(b.decompress(pb, ctx)))
    gathered_u8 = torch.cat([pa[0], pa[0], ops.sign_encode(-x)])
    gathered_bits = torch.cat([pb[0], pb[0], ops.pack_bits(ops.sign_encode(-x))])
    assert same_bits(_np(a.decode_aggregate_gathered([gathered_u8], ctx, 3)),
                     _np(b.decode_aggregate_gathered([gathered_bits], ctx, 3)))
    t8, t2 = TernGradCompressor(), TernGradCompressor(wire="2bit")
    p8, ctx = t8.compress(x, "w")
    p2, _ = t2.compress(x, "w")          # same step seed -> same codes
    assert p2[0].numel() == (x.numel() + 4 - x.numel() % 4) // 4
    assert same_bits(_np(t8.decompress(p8, ctx)), _np(t2.decompress(p2, ctx)))
