"""GPU parity at the two BASELINE configurations whose code paths only run at full size.

configs[2]: QSGD(127, 128) and TernGrad over the whole 161-tensor ResNet-50 gradient set
(25,557,032 elements, 199,672 QSGD buckets) in one segmented launch per stage.  At this size the
QSGD encoder grid is capped (4096 workgroups x 32 buckets per pass, csrc/quant.hip), so every
workgroup walks its bucket range more than once -- the path no smaller test reaches.  Checked per
segment against the oracle (which restates grace_dl/dist/compressor/qsgd.py:12-49 and
terngrad.py:7-30): codewords bit-exact given the same uniforms and scales, device scales within
4 ulp of torch's CPU f32 reductions, decode bit-exact.

configs[4]: ShardedTopK(0.001) with W = 8 ranks on a 2^26-element (256 MiB) bucket.  The ranks
share cuda:0 over gloo (RCCL needs one device per rank; the 8-GPU RCCL run is the driver's), so
the W = 8 records (capacity k = 67,108 each) and the select over their 536,864 entries run
natively.  The union of the payloads, the residual shards and the replicated dense output are
compared with the oracle's whole-bucket top-k + residual step (grace_dl/dist/compressor/
topk.py:32-42, memory/residual.py:10-20).  A second, tie-heavy W = 8 case (99.95 % zeros) sends
thousands of tied zeros through the select's boundary ranking.
"""
import hashlib
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.detach().cpu().numpy()


def resnet50_sizes():
    import bench
    return [int(np.prod(s)) for s in bench.resnet50_shapes()]


@pytest.fixture(scope="module")
def resnet_set():
    sizes = resnet50_sizes()
    assert len(sizes) == 161 and sum(sizes) == 25_557_032
    rng = np.random.default_rng(3)
    xs = [(rng.standard_normal(n, dtype=np.float32) * np.float32(0.01)).astype(np.float32) for n in sizes]
    u = rng.random(sum(sizes), dtype=np.float32)
    return sizes, xs, u


def test_resnet50_set_qsgd_full(resnet_set):
    from grace_amd import ops
    sizes, xs, u = resnet_set
    nb = sum(-(-n // 128) for n in sizes)
    assert nb == 199_672 and nb > 4096 * 32          # multi-pass encoder path
    flat = _t(np.concatenate(xs))
    du = _t(u)
    norms_or = np.concatenate([O.qsgd_norms(x, 128) for x in xs])
    # device norms: within 4 ulp of torch's f32 per-bucket reduction
    codes, norms = ops.qsgd_compress(flat, 127, 128, sizes=sizes, u=du)
    norms = _np(norms)
    assert norms.shape == (nb,)
    assert ops.isclose_f32_ulps(norms, norms_or, 4)
    # codewords given the device norms: bit-exact per segment
    codes = _np(codes)
    off = boff = 0
    exp_codes = []
    for n, x in zip(sizes, xs):
        b = -(-n // 128)
        c, _ = O.qsgd_compress(x, u[off:off + n], 127, 128, norms=norms[boff:boff + b])
        exp_codes.append(c)
        off += n
        boff += b
    assert np.array_equal(codes, np.concatenate(exp_codes))
    # codewords given the oracle's norms (norms injected): bit-exact
    codes_in, _ = ops.qsgd_compress(flat, 127, 128, sizes=sizes, u=du, norms_in=_t(norms_or))
    exp_in = []
    off = boff = 0
    for n, x in zip(sizes, xs):
        b = -(-n // 128)
        exp_in.append(O.qsgd_compress(x, u[off:off + n], 127, 128, norms=norms_or[boff:boff + b])[0])
        off += n
        boff += b
    assert np.array_equal(_np(codes_in), np.concatenate(exp_in))
    # decode: bit-exact per segment
    dec = _np(ops.qsgd_decompress(_t(codes), _t(norms), 127, 128, flat.numel(), sizes=sizes))
    exp_dec = []
    off = boff = 0
    for n, c in zip(sizes, exp_codes):
        b = -(-n // 128)
        exp_dec.append(O.qsgd_decode(c, norms[boff:boff + b], 127, 128, n))
        off += n
        boff += b
    assert same_bits(dec, np.concatenate(exp_dec))


def test_resnet50_set_terngrad_full(resnet_set):
    from grace_amd import ops
    sizes, xs, u = resnet_set
    flat = _t(np.concatenate(xs))
    du = _t(u)
    clips = np.array([O.terngrad_clip(x) for x in xs], dtype=np.float32)
    # with the reference's clamp bound injected: codewords and scalars bit-exact
    codes, scal = ops.terngrad_compress(flat, sizes=sizes, clip=_t(clips), u=du)
    codes, scal = _np(codes), _np(scal)
    off = 0
    exp_c, exp_s = [], []
    for i, (n, x) in enumerate(zip(sizes, xs)):
        c, s = O.terngrad_compress(x, u[off:off + n], clip=clips[i])
        exp_c.append(c)
        exp_s.append(s)
        off += n
    assert np.array_equal(codes, np.concatenate(exp_c))
    assert same_bits(scal, np.concatenate(exp_s))
    # device statistics: every segment's scalar within 4 ulp
    codes2, scal2 = ops.terngrad_compress(flat, sizes=sizes, u=du)
    offs = np.cumsum([0] + sizes[:-1])
    exp_s2 = np.concatenate([O.terngrad_compress(x, u[o:o + n])[1] for x, n, o in zip(xs, sizes, offs)])
    assert ops.isclose_f32_ulps(_np(scal2), exp_s2, 4)
    # decode: bit-exact per segment
    dec = _np(ops.terngrad_decompress(_t(codes), _t(scal), flat.numel(), sizes=sizes))
    exp_dec = np.concatenate([O.terngrad_decode(c, s) for c, s in zip(exp_c, exp_s)])
    assert same_bits(dec, exp_dec)


# ----------------------------------------------------------------------------------------- W = 8
def _bucket(case, n, seed):
    rng = np.random.default_rng(seed)
    if case == "normal":
        return rng.standard_normal(n, dtype=np.float32)
    g = np.zeros(n, dtype=np.float32)                  # "sparse": 99.95 % exact zeros
    hot = rng.random(n) < 0.0005
    g[hot] = rng.standard_normal(int(hot.sum()), dtype=np.float32)
    return g


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def _w8_worker(rank, world, path, outdir, n, case, ratio, steps):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded import ShardedTopK
    sizes = [n // world + (1 if r < n % world else 0) for r in range(world)]
    base = sum(sizes[:rank])
    eng = ShardedTopK(ratio)
    res = {}
    for s in range(steps):
        full = _bucket(case, n, 500 + s)
        out = eng.step(torch.from_numpy(full[base:base + sizes[rank]].copy()).cuda(), "bucket")
        v, i = eng.last_payload
        v, i = v.cpu().numpy(), i.cpu().numpy()
        keep = i >= 0
        o = out.cpu().numpy()
        res[f"outsha{s}"] = np.frombuffer(_digest(o).encode(), dtype=np.uint8)
        if rank == 0:
            res[f"out{s}"] = o
        res[f"vals{s}"] = v[keep]
        res[f"idx{s}"] = i[keep]
        res[f"pad{s}"] = np.array([int((~keep).sum()), v.size])
        res[f"res{s}"] = eng.residuals["bucket"].cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("n,case,ratio,fallback", [
    (1 << 26, "normal", 0.001, False),        # BASELINE configs[4]: 256 MiB, k = 67,108, W = 8
    (8 * 131072 + 5, "sparse", 0.001, True),  # 99.95 % zeros: the local engines take their exact fallback
])
def test_sharded_topk_w8_one_device(n, case, ratio, fallback):
    world, steps = 8, 2
    k = O.ratio_k(n, ratio)
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_w8_worker, args=(world, os.path.join(tmp, "rdv"), tmp, n, case, ratio, steps),
                 nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({key: z[key] for key in z.files})
    r_or = None
    for s in range(steps):
        g = _bucket(case, n, 500 + s)
        _, v_or, i_or, r_or, out_or = O.topk_residual_step(g, r_or, ratio)
        assert i_or.size == k
        idx = np.concatenate([o[f"idx{s}"] for o in outs]).astype(np.int64)
        vals = np.concatenate([o[f"vals{s}"] for o in outs])
        assert idx.size == k, (s, idx.size, k)
        order = np.argsort(idx)
        assert np.array_equal(idx[order], i_or.astype(np.int64)), s
        assert same_bits(vals[order], v_or), s
        assert same_bits(np.concatenate([o[f"res{s}"] for o in outs]), r_or), s
        assert same_bits(outs[0][f"out{s}"], out_or), s
        sha = bytes(outs[0][f"outsha{s}"])
        assert all(bytes(o[f"outsha{s}"]) == sha for o in outs), "replicated dense outputs differ"
        caps = {int(o[f"pad{s}"][1]) for o in outs}   # every rank's record holds the shared capacity k
        assert caps == {k}
