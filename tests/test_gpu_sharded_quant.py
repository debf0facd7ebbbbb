"""Sharded sign / fp16 / natural / cnat / QSGD (grace_amd/dist/sharded_quant.py) with the NATIVE
kernels: 2 and 3 processes share cuda:0 over gloo (RCCL needs one device per rank).  Every rank's
result is compared bit-for-bit with the single-GPU codec on the whole bucket (ops.*_compress then
*_decompress, themselves pinned against the reference in test_gpu_quant.py / test_gpu_configs.py),
with the device generator -- a shard's draws are keyed by the bucket's element index
(grace_*_compress_at), so rank 0's whole-bucket-shaped call and the other ranks' offset calls must
reproduce the single call's stream -- and with injected streams."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
F32 = np.float32
Q, BUCKET = 127, 128
# tensors of 0..4 work units, unaligned offsets, a 1-element tensor
SIZES = [64, 16384, 100003, 1, 2048, 16385, 40000, 7, 65536, 3001]


def _data(seed, sizes=SIZES):
    rng = np.random.default_rng(seed)
    flat = np.concatenate([(rng.standard_normal(n) * (0.01 * (1 + i % 3))).astype(F32) for i, n in enumerate(sizes)])
    flat[11] = F32(-0.0)
    u = rng.random(flat.size).astype(F32)
    ri = rng.integers(0, 2 ** 23 - 1, flat.size).astype(np.int32)
    return flat, u, ri


def _stream(codec, use_u, u, ri):
    if not use_u:
        return None
    return ri if codec == "natural" else u


def _worker(rank, world, path, outdir, codec, dense, use_u, det, q, sizes=SIZES):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded_quant import ShardedQuant
    codec, _, wire = codec.partition(":")   # "sign:u8": the u8 wire instead of the 1-bit default
    eng = ShardedQuant(codec, dense=dense, quantum_num=q, bucket_size=BUCKET, deterministic=det, seed=13,
                       wire=wire or None)
    flat, u, ri = _data(4, sizes)
    lo, hi = eng.partition(sizes)[rank]
    s = _stream(codec, use_u, u, ri)
    res = {"lo": np.array([lo, hi])}
    for step in range(2):   # two steps: the plan is reused
        x = torch.from_numpy(flat[lo:hi] * F32(step + 1)).cuda()
        out = eng.step(x, sizes, u=torch.from_numpy(s[lo:hi].copy()).cuda() if s is not None else None)
        res[f"out{step}"] = out.cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _single(codec, x, s, det, q, sizes=SIZES):
    from grace_amd import ops
    codec = codec.partition(":")[0]
    n = x.numel()
    if codec == "sign":
        return ops.sign_decode(ops.sign_encode(x))
    if codec == "fp16":
        return ops.fp16_decompress(ops.fp16_compress(x))
    if codec == "natural":
        return ops.natural_decompress(ops.natural_compress(x, rand_int=s, seed=13), n, 0)
    if codec == "cnat":
        return ops.natural_decompress(ops.cnat_compress(x, rand=s, deterministic=det, seed=13), n, 1)
    codes, norms = ops.qsgd_compress(x, q, BUCKET, sizes=sizes, u=s, seed=13)
    return ops.qsgd_decompress(codes, norms, q, BUCKET, n, sizes=sizes)


def _oracle(codec, xv, s, det, q, sizes=SIZES, norms=None):
    """The reference restatement (oracle/grace_oracle.py) on the whole bucket, where it is fully
    determined: the deterministic codecs, and the stochastic ones with the injected stream (QSGD
    tensor by tensor, every bucket counted from its tensor's start, with the device's bucket norms
    injected: the parity bar is bit-exact codewords given the reference's u and norm, the norms
    themselves within 4 ulp of torch's f32 reduction, test_gpu_quant.py); None otherwise."""
    from oracle import grace_oracle as O
    codec = codec.partition(":")[0]
    if codec == "sign":
        return O.sign_decode(O.sign_encode(xv))
    if codec == "fp16":
        return O.fp16_decode(O.fp16_compress(xv))
    if codec == "natural":
        return O.natural_decode(O.natural_compress(xv, s)) if s is not None else None
    if codec == "cnat":
        return O.cnat_decode(O.cnat_compress(xv, None if det else s)) if (det or s is not None) else None
    if s is None or q >= 128:
        return None
    out, a, b = [], 0, 0
    for n in sizes:
        nb = -(-n // BUCKET)
        c, nm = O.qsgd_compress(xv[a:a + n], s[a:a + n], q, BUCKET, norms=norms[b:b + nb])
        out.append(O.qsgd_decode(c, nm, q, BUCKET, n))
        a += n
        b += nb
    return np.concatenate(out)


def _bits(a, b):
    return np.array_equal(np.asarray(a, F32).view(np.uint32), np.asarray(b, F32).view(np.uint32))


CASES = [("sign", False, False, Q), ("sign:u8", False, False, Q), ("fp16", False, False, Q), ("natural", False, False, Q),
         ("natural", True, False, Q), ("cnat", False, False, Q), ("cnat", True, False, Q), ("cnat", False, True, Q),
         ("qsgd", False, False, Q), ("qsgd", True, False, Q), ("qsgd", False, False, 255)]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("codec,use_u,det,q", CASES)
@pytest.mark.parametrize("dense", ["replicated", "shard"])
def test_sharded_quant_native_matches_single_gpu(world, codec, use_u, det, q, dense):
    if dense == "shard" and world == 3 and codec in ("sign", "sign:u8", "fp16"):
        pytest.skip("covered by world 2 (deterministic codecs)")
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, codec, dense, use_u, det, q), nprocs=world,
                 join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    flat, u, ri = _data(4)
    s = _stream(codec, use_u, u, ri)
    for step in range(2):
        x = torch.from_numpy(flat * F32(step + 1)).cuda()
        exp = _single(codec, x, torch.from_numpy(s).cuda() if s is not None else None, det, q).cpu().numpy()
        norms = None
        if codec == "qsgd" and s is not None:
            from grace_amd import ops
            norms = ops.qsgd_compress(x, q, BUCKET, sizes=SIZES, u=torch.from_numpy(s).cuda(), seed=13)[1].cpu().numpy()
        ref = _oracle(codec, flat * F32(step + 1), s, det, q, norms=norms)
        if ref is not None:   # the native result against the reference restatement directly too
            assert _bits(exp, np.asarray(ref, F32)), (step, codec, "single-GPU codec vs oracle")
            for o in outs:
                if dense == "replicated":
                    assert _bits(o[f"out{step}"], np.asarray(ref, F32)), (step, codec, "sharded vs oracle")
        if dense == "shard":
            assert _bits(np.concatenate([o[f"out{step}"] for o in outs]), exp), (step, codec)
        else:
            for o in outs:
                assert _bits(o[f"out{step}"], exp), (step, codec)
    assert int(outs[0]["lo"][0]) == 0 and int(outs[-1]["lo"][1]) == flat.size


@pytest.mark.parametrize("codec", ["sign", "qsgd"])
@pytest.mark.parametrize("dense", ["replicated", "shard"])
def test_sharded_quant_native_rank_without_elements(codec, dense):
    """A bucket of fewer partition units than ranks (one 128-element block; two QSGD buckets) over 3
    processes: the last rank's shard is empty, it still joins the all-gather, and every rank's result
    equals the single-GPU codec's."""
    sizes = [100] if codec == "sign" else [130]
    world = 3
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, codec, dense, False, False, Q, sizes),
                 nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    assert int(outs[-1]["lo"][0]) == int(outs[-1]["lo"][1])
    flat, _, _ = _data(4, sizes)
    for step in range(2):
        x = torch.from_numpy(flat * F32(step + 1)).cuda()
        exp = _single(codec, x, None, False, Q, sizes).cpu().numpy()
        if dense == "shard":
            assert _bits(np.concatenate([o[f"out{step}"] for o in outs]), exp), step
        else:
            for o in outs:
                assert _bits(o[f"out{step}"], exp), step
