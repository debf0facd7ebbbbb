"""CPU oracle for the grace_amd gradient-codec hot path.

TEST INFRASTRUCTURE ONLY.  This module is a CPU restatement of the reference
codecs (sands-lab/grace ``grace_dl/dist``) with every source of randomness and
every data-dependent scale made an explicit argument, so that the HIP kernels
can be checked bit-for-bit.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``grace_amd``) never does.

Pinning: every function is checked against golden vectors produced by running
the reference itself in the build container (tests/golden/gen_golden.py ->
tests/golden/*.npz; tests/test_oracle_golden.py).  Exceptions, marked
"parity unpinned" below: the cupy ``NaturalCompressor`` (cupy 8.2.0 pinned at
environment.yml:17 is absent here) and the ``cnat_cuda`` / ``qsgd_cuda`` CUDA
extensions (no nvcc / GPU); those are restated from their source text.

Floating-point reductions (means, norms, std) use torch CPU ops in the same
order as the reference so the oracle reproduces the fixtures exactly; bit and
integer work is numpy.
"""
import math

import numpy as np
import torch

F32 = np.float32


def _f32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=F32))


def abs_key(x):
    """uint32 ordering key of |x|: monotone in |x|, NaN above +inf, -0 == +0."""
    return _f32(x).view(np.uint32) & np.uint32(0x7FFFFFFF)


def ratio_k(numel, ratio):
    """k = max(1, int(numel * ratio))  (grace_dl/dist/compressor/topk.py:34, randomk.py:9)."""
    return max(1, int(numel * ratio))


def python_sum(arrays):
    """Python ``sum(list)`` as used by Compressor.aggregate (grace_dl/dist/__init__.py:32-34):
    ``((0 + d0) + d1) + ...`` in f32 (0 + -0.0 -> +0.0)."""
    acc = None
    for a in arrays:
        a = _f32(a)
        acc = (F32(0) + a) if acc is None else (acc + a)
    return acc.astype(F32)


# ----------------------------------------------------------------------------- sign family
def sign_encode(x):
    """signSGD codeword: uint8 (x >= 0); -0 -> 1, NaN -> 0 (signsgd.py:15-16)."""
    return (_f32(x).ravel() >= 0).astype(np.uint8)


def sign_decode(codes):
    """u8 * 2 - 1 in f32 (signsgd.py:21)."""
    return (codes.astype(F32) * F32(2) - F32(1)).astype(F32)


def sign_aggregate(decoded):
    """majority vote: sum >= 0 -> +1 else -1 (signsgd.py:25-30)."""
    s = python_sum(decoded)
    return ((s >= 0).astype(F32) * F32(2) - F32(1)).astype(F32)


def signum_momentum(x, prev, momentum):
    """m = (1-beta) g + beta m_prev (signum.py:19-21); first step m = g."""
    x = torch.from_numpy(_f32(x).ravel().copy())
    if prev is None:
        return x.numpy()
    prev = torch.from_numpy(_f32(prev).ravel().copy())
    return ((1.0 - momentum) * x + momentum * prev).numpy()


def efsign_compress(t):
    """(mean|t|, u8 signs)  (efsignsgd.py:17-19)."""
    tt = torch.from_numpy(_f32(t).ravel().copy())
    mean = tt.abs().mean().numpy().reshape(1)
    return mean.astype(F32), sign_encode(t)


def efsign_decode(mean, codes):
    """mean * (2 s - 1)  (efsignsgd.py:26-27)."""
    return (F32(mean.reshape(())) * sign_decode(codes)).astype(F32)


def efsign_compensate(g, residual, lr):
    """t = r + lr * g, first step t = g (grace_dl/dist/memory/efsignsgd.py:11-13)."""
    if residual is None:
        return _f32(g).copy()
    return (torch.from_numpy(_f32(residual).copy()) + lr * torch.from_numpy(_f32(g).copy())).numpy()


def onebit_compress(x):
    """(mask0 = x<0 as u8, mean0, mean1)  (onebit.py:13-23)."""
    t = torch.from_numpy(_f32(x).ravel().copy())
    mask0 = t < 0
    sum0 = torch.sum(t[mask0])
    num0 = torch.sum(mask0).float()
    mean0 = sum0 / num0 if num0 > 0 else sum0
    mask1 = ~mask0
    sum1 = torch.sum(t[mask1])
    num1 = t.numel() - num0
    mean1 = sum1 / num1 if num1 > 0 else sum1
    return mask0.numpy().astype(np.uint8), F32(mean0.item()), F32(mean1.item())


def onebit_decode(mask0, mean0, mean1, quirk=False):
    """Fixed semantics (grace_dl/torch/compressor/onebit.py:29) by default; ``quirk=True``
    reproduces the dist flavour's uint8 ``~`` (onebit.py:29: ~1 = 254, ~0 = 255)."""
    m = mask0.astype(F32)
    notm = (np.uint8(255) - mask0).astype(F32) if quirk else (F32(1) - m)
    return (m * F32(mean0) + notm * F32(mean1)).astype(F32)


# ----------------------------------------------------------------------------- sparsifiers
def topk_select(x, k):
    """Exact top-k of |x| with a deterministic tie rule: larger |x| first (NaN largest), and
    among equal |x| the lower index first.  Returns (values f32[k], indices int32[k]) sorted by
    index.  torch.topk(sorted=False) (topk.py:36) returns the same set modulo ties at the k-th
    value; the HIP kernels implement exactly this rule."""
    xf = _f32(x).ravel()
    n = xf.size
    key = abs_key(xf)
    if k >= n:
        idx = np.arange(n, dtype=np.int64)
    else:
        # k-th largest key, then everything above it plus the lowest-index ties
        kth = np.partition(key, n - k)[n - k]
        above = np.nonzero(key > kth)[0]
        ties = np.nonzero(key == kth)[0][: k - above.size]
        idx = np.sort(np.concatenate([above, ties]))
    return xf[idx].copy(), idx.astype(np.int32)


def sparse_decode(vals, idx, numel):
    """zeros(numel).scatter_(idx, vals)  (topk.py:45-49, randomk.py:39-40, threshold.py:25-26)."""
    out = np.zeros(numel, dtype=F32)
    out[np.asarray(idx, dtype=np.int64)] = _f32(vals)
    return out


def residual_compensate(g, residual, beta=1.0, gamma=1.0):
    """t = beta r + gamma g; first step t = g (grace_dl/dist/memory/residual.py:10-14)."""
    g = torch.from_numpy(_f32(g).copy())
    if residual is None:
        return g.numpy()
    return (beta * torch.from_numpy(_f32(residual).copy()) + gamma * g).numpy()


def residual_update(t, decoded):
    """r' = t - decompress(compress(t))  (residual.py:16-20)."""
    return (_f32(t).ravel() - _f32(decoded).ravel()).astype(F32)


def topk_residual_step(g, residual, ratio, world_size=1):
    """One Allgather(TopK, ResidualMemory, 1).step on a flat bucket (world 1).
    Returns (t, vals, idx, new_residual, out)."""
    t = residual_compensate(g, residual).ravel()
    k = ratio_k(t.size, ratio)
    vals, idx = topk_select(t, k)
    dec = sparse_decode(vals, idx, t.size)
    new_res = residual_update(t, dec)
    out = (python_sum([dec]) / F32(world_size)).astype(F32)
    return t, vals, idx, new_res, out


def randomk_indices(name, step, numel, ratio):
    """torch.manual_seed(sum(bytes(name)) + step); randint(numel, [k])  (randomk.py:11,27-29).
    Note: like the reference this reseeds torch's global generator."""
    h = sum(bytes(name, encoding="utf8"), step)
    torch.manual_seed(h)
    return torch.randint(numel, [ratio_k(numel, ratio)]).numpy(), h


def randomk_decode(vals, idx, numel):
    """zeros.scatter_(idx, vals): duplicates resolve to the last write in index order
    (CPU scatter_ is sequential; randomk.py:39-40)."""
    out = np.zeros(numel, dtype=F32)
    for i, v in zip(np.asarray(idx, dtype=np.int64), _f32(vals)):
        out[i] = v
    return out


def threshold_select(x, thr):
    """idx = where(|x| >= min(thr, max(x))) (signed max; threshold.py:16).  Python ``min``
    returns thr when max(x) is NaN; the compare runs in f32."""
    xf = _f32(x).ravel()
    mx = F32(np.max(xf)) if not np.isnan(xf).any() else F32(np.nan)
    bound = mx if (mx < F32(thr)) else F32(thr)
    idx = np.nonzero(np.abs(xf) >= bound)[0]
    return xf[idx].copy(), idx.astype(np.int32)


# ----------------------------------------------------------------------------- TernGrad
def terngrad_clip(x):
    """c = 2.5 * std(x) as a Python double, std = sqrt(mean((x - mean x)^2)) in f32 torch
    order (terngrad.py:11-13).  Returned as the f32 clamp bound."""
    t = torch.from_numpy(_f32(x).ravel().copy())
    std = torch.sqrt(torch.mean((t - torch.mean(t)) ** 2))
    return F32(2.5 * std.item())


def terngrad_compress(x, u, clip=None):
    """TernGrad codeword with injected uniforms ``u`` (terngrad.py:14-24).
    Returns (codes int8[n], scalar f32[1])."""
    xf = _f32(x).ravel()
    c = terngrad_clip(xf) if clip is None else F32(clip)
    clamped = np.minimum(np.maximum(xf, -c), c).astype(F32)
    # torch.clamp propagates NaN; numpy min/max also propagate NaN
    absg = np.abs(clamped)
    scalar = F32(np.max(absg)) if absg.size else F32(0)
    rnd = (_f32(u).ravel() * scalar).astype(F32)
    keep = ~(rnd >= absg)
    codes = np.where(keep, np.sign(clamped) * (scalar != 0), 0).astype(np.int8)
    return codes, np.array([scalar], dtype=F32)


def terngrad_decode(codes, scalar):
    return (codes.astype(F32) * F32(scalar.reshape(-1)[0])).astype(F32)


# ----------------------------------------------------------------------------- QSGD
def qsgd_norms(x, bucket_size):
    """Per-bucket L2 norms over the zero-padded tensor, f32 torch order (qsgd.py:17-24)."""
    t = torch.from_numpy(_f32(x).ravel().copy())
    n = t.numel()
    if n % bucket_size:
        t = torch.cat([t, torch.zeros(bucket_size - n % bucket_size)])
    return torch.sqrt(torch.sum(t.view(-1, bucket_size) ** 2, dim=1)).numpy()


def _f2int16_x86(v):
    """float -> int16 as torch CPU does on x86 (cvttss2si to int32, keep the low 16 bits):
    NaN and |v| >= 2^31 give 0x80000000 -> 0."""
    v = np.asarray(v, dtype=np.float64)
    bad = ~np.isfinite(v) | (np.abs(v) >= 2.0 ** 31)
    iv = np.where(bad, 0, np.trunc(np.where(bad, 0, v))).astype(np.int64)
    return (iv & 0xFFFF).astype(np.uint16).view(np.int16)


def qsgd_compress(x, u, quantum_num, bucket_size, norms=None):
    """QSGD codeword with injected uniforms and (optionally) injected bucket norms
    (qsgd.py:12-39).  ``q / norm`` is torch's ``Tensor.__rdiv__`` = reciprocal(norm) * q."""
    xf = _f32(x).ravel()
    n = xf.size
    if norms is None:
        norms = qsgd_norms(xf, bucket_size)
    norms = _f32(norms)
    norm = np.repeat(norms, bucket_size)[:n]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        recip = (F32(1) / norm).astype(F32)
        level = ((recip * F32(quantum_num)).astype(F32) * np.abs(xf)).astype(F32)
        prev = np.floor(level).astype(F32)
        nxt = (_f32(u).ravel() < (level - prev).astype(F32)).astype(F32)
        new_level = (prev + nxt).astype(F32)
        signed = (new_level * np.sign(xf).astype(F32)).astype(F32)
    i16 = _f2int16_x86(signed)
    if quantum_num < 128:
        codes = i16.astype(np.int8)
    else:
        codes = i16.astype(np.float16)
    return codes, norms


def qsgd_decode(codes, norms, quantum_num, bucket_size, numel):
    """(norm / q) * code  (qsgd.py:44-49)."""
    norm = np.repeat(_f32(norms), bucket_size)[:numel]
    return ((norm / F32(quantum_num)).astype(F32) * codes.astype(F32)).astype(F32)


def qsgd_cuda_compress(x, u, quantum_num, bucket_size, norms=None):
    """qsgd_cuda restatement (qsgd_cuda.cu:320-388): f64 bucket norms over finite elements,
    level = (float)level / (float)norm * |x|, NaN/Inf -> -128.  Parity unpinned (CUDA only).
    ``norms`` (optional) injects the bucket norms, as qsgd_compress does."""
    xf = _f32(x).ravel()
    n = xf.size
    nb = -(-n // bucket_size)
    fin = np.isfinite(xf)
    if norms is None:
        norms = np.zeros(nb, dtype=np.float64)
        xd = np.where(fin, xf.astype(np.float64), 0.0)
        np.add.at(norms, np.arange(n) // bucket_size, xd * xd)
        norms = np.sqrt(norms)
    else:
        norms = np.asarray(norms, dtype=np.float64)
    nsc = norms.astype(F32)[np.arange(n) // bucket_size]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        lf = ((F32(quantum_num) / nsc).astype(F32) * np.abs(xf)).astype(F32)
        prev = np.floor(lf)
        lvl = prev + (_f32(u).ravel() < (lf - prev)).astype(F32)
        codes = np.where(xf < 0, -lvl, lvl)
    ok = np.isfinite(nsc) & fin
    codes = np.where(ok, np.nan_to_num(codes), -128).astype(np.int64).astype(np.int8)
    return codes, norms


# ----------------------------------------------------------------------------- Horovod flavour
def qsgd_global_compress(x, u, quantum_num, norm=None):
    """grace_dl/torch/compressor/qsgd.py:12-31: ONE norm ``tensor.norm()`` over the whole tensor, then
    the dist codeword rule.  Returns (codes, norm f32[1])."""
    xf = _f32(x).ravel()
    if norm is None:
        norm = np.array([torch.from_numpy(xf.copy()).norm().item()], dtype=F32)
    norm = _f32(norm).reshape(1)
    codes, _ = qsgd_compress(xf, u, quantum_num, max(xf.size, 1), norms=norm)
    return codes, norm


def qsgd_global_decode(codes, norm, quantum_num, numel):
    """norm / q * code (grace_dl/torch/compressor/qsgd.py:33-38)."""
    return qsgd_decode(codes, _f32(norm).reshape(1), quantum_num, max(numel, 1), numel)


def threshold_select_strict(x, thr):
    """grace_dl/torch/compressor/threshold.py:17: where(|x| > thr) with thr rounded to f32 (torch
    compares a float32 tensor with a Python scalar in float32); int64 indices."""
    xf = _f32(x).ravel()
    with np.errstate(invalid="ignore"):
        idx = np.nonzero(np.abs(xf) > F32(thr))[0]
    return xf[idx].copy(), idx.astype(np.int64)


def randomk_perm_indices(name, step, numel, ratio):
    """grace_dl/torch/compressor/randomk.py:6-29: manual_seed(sum(bytes(name)) + step), then
    randperm(numel)[:k] (no replacement)."""
    h = sum(bytes(name, encoding="utf8"), step)
    torch.manual_seed(h)
    return torch.randperm(numel)[:ratio_k(numel, ratio)].numpy(), h


# ----------------------------------------------------------------------------- natural
def natural_compress(x, rnd_int):
    """cupy NaturalCompressor restated bit-for-bit (grace_dl/dist/compressor/natural.py:12-29),
    with the ``randint(0, 2^23-1)`` stream injected.  Parity unpinned (cupy absent)."""
    bits = _f32(x).ravel().view(np.int32)
    sign = bits & np.int32(-2 ** 31)
    exp = bits & np.int32(0x7F800000)
    mant = bits & np.int32(0x007FFFFF)
    up = mant > np.asarray(rnd_int, dtype=np.int32).ravel()
    e = np.where(up, exp + np.int32(0x00800000), exp)
    e = np.clip(e, np.int32(0x09000000), np.int32(0x48800000))
    code = np.bitwise_or(np.right_shift(sign, 24), np.right_shift(e, 23) - 18)
    return code.astype(np.uint8)


def natural_decode(codes):
    """(natural.py:35-39): +-2^(c&0x7f + 18 - 127), c&0x7f == 0 -> +-0 (0x80 -> -0.0)."""
    c = np.asarray(codes, dtype=np.uint8)
    e = (c & 0x7F).astype(np.int32)
    mag = ((e + 18) << 23).astype(np.int32).view(F32)
    val = np.where(c > 127, -mag, mag).astype(F32)
    return (val * (e >= 1).astype(F32)).astype(F32)


def cnat_compress(x, rand=None):
    """cnat_cuda restated (cnat_cuda.cu:68-123): frexp mantissa m in [0.5,1); keep exponent w.p.
    2|m|-1 (rand >= prob -> exp-1); LUT: biased E <= 17 -> 0, E -> E-17 saturating at 127, +128
    for negatives.  ``rand=None`` is compress_deterministic (threshold 0.5).  Parity unpinned."""
    xf = _f32(x).ravel()
    m, e = np.frexp(xf)
    prob = (np.abs(m).astype(F32) / F32(0.5) - F32(1)).astype(F32)
    thr = F32(0.5) if rand is None else _f32(rand).ravel()
    e = np.where(thr >= prob, e - 1, e).astype(np.int64)
    biased = e + 127
    code = np.where(biased <= 17, 0, np.minimum(biased - 17, 127))
    code = np.where(xf < 0, code + 128, code)
    code = np.where(xf == 0, 0, code)
    return code.astype(np.uint8)


def cnat_decode(codes):
    """encoding_to_sign_and_exp (cnat_cuda.cu:47-66, 125-134): c -> sign|E=c+17, 0 -> +0,
    128 -> -0."""
    c = np.asarray(codes, dtype=np.int64)
    mag = c & 0x7F
    e = np.where(mag == 0, 0, mag + 17)
    word = ((c >> 7) << 31) | (e << 23)
    return (word & 0xFFFFFFFF).astype(np.uint32).view(F32)


# ----------------------------------------------------------------------------- PowerSGD
def orthogonalize(a):
    """Modified Gram-Schmidt in place on columns (powersgd.py:7-18), f32 torch ops."""
    mat = torch.from_numpy(_f32(a).copy())
    n, m = mat.shape
    for i in range(m):
        col = mat[:, i:i + 1]
        col /= torch.sqrt(torch.sum(col ** 2))
        if i + 1 < m:
            rest = mat[:, i + 1:]
            rest -= torch.sum(col * rest, dim=0) * col
    return mat.numpy()


def powersgd_compress(x2d, q, world_size=1):
    """P = M q, orthogonalize P, Q = M^T P (powersgd.py:45-52), world 1 (all_reduce = id)."""
    mat = torch.from_numpy(_f32(x2d).copy())
    p = torch.mm(mat, torch.from_numpy(_f32(q).copy())) / world_size
    p = torch.from_numpy(orthogonalize(p.numpy()))
    qq = torch.mm(mat.t(), p) / world_size
    return p.numpy(), qq.numpy()


def powersgd_decode(p, q):
    return torch.mm(torch.from_numpy(_f32(p)), torch.from_numpy(_f32(q)).t()).numpy()


# ----------------------------------------------------------------------------- fp16
def fp16_compress(x):
    return _f32(x).astype(np.float16)


def fp16_decode(h):
    return np.asarray(h, dtype=np.float16).astype(F32)


def bucket_gbps(numel, seconds):
    """Headline unit: 4 n bytes of f32 bucket per second, in GB/s."""
    return 4.0 * numel / seconds / 1e9


__all__ = [n for n in dir() if not n.startswith("_")] + ["math"]


# ------------------------------------------------------------------------------------------ DGC
def dgc_compress(x, sample_idx, ratio):
    """DgcCompressor.compress (grace_dl/dist/compressor/dgc.py:12-43) given the sampled indices
    (torch.empty(ns).uniform_(0, numel).long()).  Returns (values f32, indices int64, mask, thr).
    thr0 = min of the k_s largest |sample| (torch.topk puts NaN first; torch.min propagates NaN);
    each adjustment is f32(1.3) * thr / f32(0.7) * thr, and the count is compared with the
    Python double 1.3 * numel * ratio in f32 (torch promotes the int64 count with a float
    scalar to the default dtype)."""
    t = _f32(x).ravel()
    numel = t.size
    s = np.abs(t[np.asarray(sample_idx, dtype=np.int64)]).astype(F32)
    k = max(1, int(numel * ratio * 0.01))
    key = np.where(np.isnan(s), np.inf, s)
    order = np.argsort(-key, kind="stable")
    top = s[order[:k]]
    thr = F32(np.min(top)) if not np.isnan(top).any() else F32(np.nan)
    a = np.abs(t)
    hi = F32(1.3 * numel * ratio)
    lo = F32(0.7 * numel * ratio)
    mask = a >= thr
    sel = F32(mask.sum())
    for _ in range(10):
        if sel > hi:
            thr = F32(F32(1.3) * thr)
        elif sel < lo:
            thr = F32(F32(0.7) * thr)
        else:
            break
        mask = a >= thr
        sel = F32(mask.sum())
    idx = np.nonzero(mask)[0].astype(np.int64)
    return t[idx].copy(), idx, mask, thr


def dgc_memory_compensate(g, residual, accum, momentum):
    """DgcMemory.compensate without clipping (memory/dgc.py:20-29): r = m r + g; a = a + r
    (first step r = a = g).  Returns (t, r, a)."""
    g = _f32(g).ravel()
    if residual is None:
        return g.copy(), g.copy(), g.copy()
    r = (F32(momentum) * _f32(residual) + g).astype(F32)
    a = (_f32(accum) + r).astype(F32)
    return a.copy(), r, a


def dgc_memory_update(residual, accum, mask):
    """DgcMemory.update (memory/dgc.py:31-39): r * ~mask, a * ~mask (f32 multiply by 0/1)."""
    keep = (~np.asarray(mask, dtype=bool)).astype(F32)
    return (_f32(residual) * keep).astype(F32), (_f32(accum) * keep).astype(F32)


# ------------------------------------------------------------------------------------------ AllToAll
def alltoall_two_phase(grads, kind, u1, u2, quantum_num=127, bucket_size=128, average=True):
    """AllToAll.send_receive (grace_dl/dist/communicator/all_to_all.py:29-124) for all W ranks at
    once, with ZERO padding (the reference pads with torch.empty: uninitialised, see
    grace_amd/dist/communicator/all_to_all.py).  grads[r]: rank r's gradient; u1[r] / u2[r]: the
    uniforms of rank r's compress of its whole tensor and of its aggregated chunk.
    kind 'qsgd' | 'terngrad'.  Returns the per-rank outputs (identical on every rank).
    Parity of the communicator is unpinned (gloo has no list all_to_all, so the reference cannot
    run here); the codecs it composes are pinned by their own golden vectors."""
    W = len(grads)
    n = _f32(grads[0]).size
    unit = W * bucket_size if kind == "qsgd" else W
    n_pad = -(-n // unit) * unit
    chunk = n_pad // W

    def compress(x, u):
        if kind == "qsgd":
            return qsgd_compress(x, u, quantum_num, bucket_size)
        return terngrad_compress(x, u)

    def decode(payload, numel):
        if kind == "qsgd":
            return qsgd_decode(payload[0], payload[1], quantum_num, bucket_size, numel)
        return terngrad_decode(payload[0], payload[1])

    pay = [compress(grads[r], u1[r]) for r in range(W)]
    codes_p = [np.concatenate([p[0], np.zeros(n_pad - n, dtype=p[0].dtype)]) for p in pay]
    agg = []
    for r in range(W):       # rank r's chunk
        decs = []
        for w in range(W):
            c = codes_p[w][r * chunk:(r + 1) * chunk]
            if kind == "qsgd":
                nb = chunk // bucket_size
                norms = np.concatenate([pay[w][1], np.zeros(n_pad // bucket_size - pay[w][1].size, F32)])
                decs.append(qsgd_decode(c, norms[r * nb:(r + 1) * nb], quantum_num, bucket_size, chunk))
            else:
                decs.append(terngrad_decode(c, pay[w][1]))
        agg.append(python_sum(decs))
    pay2 = [compress(agg[r], u2[r]) for r in range(W)]
    full = np.concatenate([decode(pay2[r], chunk) for r in range(W)])[:n]
    if average:
        full = (full / F32(W)).astype(F32)
    return full


# ------------------------------------------------------------------------------------------ wire formats
def pack2_encode(values):
    """grace_dl/tensorflow/compressor/packing.py:4-17 encode_byte: pad with range(0, 4 - n % 4)
    (4 values when n % 4 == 0), split into 4 planar quarters, byte = a1 + 4 a2 + 16 a3 + 64 a4.
    TensorFlow is absent here: restated from source, parity unpinned."""
    a = np.asarray(values, dtype=np.int64).ravel()
    pad = 4 - a.size % 4
    a = np.concatenate([a, np.arange(pad, dtype=np.int64)])
    q = a.size // 4
    s = a[:q] + a[q:2 * q] * 4 + a[2 * q:3 * q] * 16 + a[3 * q:] * 64
    return s.astype(np.uint8)


def pack2_decode(encoded, real_size):
    """packing.py:20-29 decode_byte."""
    a = np.asarray(encoded, dtype=np.int64)
    parts = [a % 4, (a // 4) % 4, (a // 16) % 4, (a // 64) % 4]
    return np.concatenate(parts)[:real_size].astype(np.int32)
