"""Tensor-level wrappers over the C ABI.

Every function takes torch tensors that live on the GPU (torch provides device memory and the
current HIP stream only; all arithmetic runs in libgrace_hip.so), validates dtype / contiguity,
allocates outputs and launches on ``torch.cuda.current_stream()``.
"""
import math

import torch

from . import _lib

F32 = torch.float32


class GraceDeviceError(TypeError):
    """A grace_amd codec was handed a tensor that is not on the GPU."""


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return t.data_ptr() if t is not None else None


def dev_f32(t, what="tensor"):
    """Flat, contiguous f32 device view of t (no copy when already so)."""
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise GraceDeviceError(
            f"grace_amd: {what} must be a GPU tensor (MI355X); got "
            f"{getattr(t, 'device', type(t))}. There is no CPU path.")
    if t.dtype != F32:
        raise TypeError(f"grace_amd: {what} must be float32, got {t.dtype}")
    return t.reshape(-1) if t.is_contiguous() else t.contiguous().reshape(-1)


def require_dev(t, what="tensor"):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise GraceDeviceError(f"grace_amd: {what} must be a GPU tensor; got {getattr(t, 'device', type(t))}")
    return t.contiguous()


# ----------------------------------------------------------------------------- workspaces
_ws = {}


def workspace(slot, nbytes, device):
    """Per-(device, slot) scratch buffer, grown on demand and reused across calls.  Reuse is safe
    because every use is ordered on the current stream."""
    key = (str(device), slot, torch.cuda.current_stream(device).cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        # zeroed once: the codecs leave their counters / histograms zeroed after every use
        buf = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


# ----------------------------------------------------------------------------- elementwise
def axpby(r, g, beta, gamma, out=None):
    r, g = dev_f32(r, "residual"), dev_f32(g, "gradient")
    out = torch.empty_like(g) if out is None else out
    _lib.call("grace_axpby", _p(r), _p(g), float(beta), float(gamma), _p(out), g.numel(), _stream())
    return out


def sub(t, d, out=None):
    t, d = dev_f32(t), dev_f32(d)
    out = torch.empty_like(t) if out is None else out
    _lib.call("grace_sub", _p(t), _p(d), _p(out), t.numel(), _stream())
    return out


def div_scalar(x, divisor, out=None):
    x = dev_f32(x)
    out = torch.empty_like(x) if out is None else out
    _lib.call("grace_div_scalar", _p(x), float(divisor), _p(out), x.numel(), _stream())
    return out


def fill(x, value):
    _lib.call("grace_fill", _p(x), float(value), x.numel(), _stream())
    return x


def sum_rank_order(tensors):
    """Python ``sum(list)`` = ((0 + t0) + t1) + ... on the device (grace_dl/dist/__init__.py:32-34)."""
    first = dev_f32(tensors[0])
    acc = torch.empty_like(first)
    for i, t in enumerate(tensors):
        t = dev_f32(t)
        _lib.call("grace_accumulate", _p(acc), _p(t), t.numel(), 1 if i == 0 else 0, _stream())
    return acc


# ----------------------------------------------------------------------------- sign family
def sign_encode(x):
    x = dev_f32(x)
    codes = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
    _lib.call("grace_sign_encode", _p(x), _p(codes), x.numel(), _stream())
    return codes


def sign_decode(codes, scale=None):
    codes = require_dev(codes, "codes")
    out = torch.empty(codes.numel(), dtype=F32, device=codes.device)
    _lib.call("grace_sign_decode", _p(codes), _p(scale) if scale is not None else None, _p(out),
              codes.numel(), _stream())
    return out


def sign_majority(codes_wn, world, n):
    codes_wn = require_dev(codes_wn, "codes")
    out = torch.empty(n, dtype=F32, device=codes_wn.device)
    _lib.call("grace_sign_majority", _p(codes_wn), int(world), _p(out), n, _stream())
    return out


def signum_encode(g, momentum_buf, has_prev, momentum):
    g = dev_f32(g)
    codes = torch.empty(g.numel(), dtype=torch.uint8, device=g.device)
    coef_g = float(torch.tensor(1.0 - momentum, dtype=F32))     # Python double, rounded as torch does
    coef_m = float(torch.tensor(momentum, dtype=F32))
    _lib.call("grace_signum_encode", _p(g), _p(momentum_buf), 1 if has_prev else 0, coef_g, coef_m,
              _p(codes), g.numel(), _stream())
    return codes


def sign_step_w1(x):
    x = dev_f32(x)
    codes = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
    out = torch.empty_like(x)
    _lib.call("grace_sign_step_w1", _p(x), _p(codes), _p(out), x.numel(), _stream())
    return codes, out


def abs_mean(x):
    x = dev_f32(x)
    out = torch.empty(1, dtype=F32, device=x.device)
    ws = workspace("reduce", _lib.query("grace_reduce_workspace_bytes", x.numel()), x.device)
    _lib.call("grace_abs_mean", _p(x), x.numel(), _p(out), _p(ws), _stream())
    return out


def onebit_encode(x):
    x = dev_f32(x)
    mask0 = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
    means = torch.empty(2, dtype=F32, device=x.device)
    ws = workspace("reduce", _lib.query("grace_reduce_workspace_bytes", x.numel()), x.device)
    _lib.call("grace_onebit_encode", _p(x), x.numel(), _p(mask0), _p(means), _p(ws), _stream())
    return mask0, means


def onebit_decode(mask0, mean0, mean1, quirk=False):
    mask0 = require_dev(mask0, "mask0")
    out = torch.empty(mask0.numel(), dtype=F32, device=mask0.device)
    _lib.call("grace_onebit_decode", _p(mask0), _p(require_dev(mean0)), _p(require_dev(mean1)),
              1 if quirk else 0, _p(out), mask0.numel(), _stream())
    return out


# ----------------------------------------------------------------------------- top-k
def ratio_k(numel, ratio):
    """k = max(1, int(numel * ratio)) (grace_dl/dist/compressor/topk.py:34)."""
    return max(1, int(numel * ratio))


def topk_workspace(n, k, device):
    return workspace("topk", _lib.query("grace_topk_workspace_bytes", n, k), device)


def new_payload(k, device):
    """One packed buffer [vals f32[k] | idx i32[k]] so the payload moves in a single collective."""
    buf = torch.empty(2 * k, dtype=F32, device=device)
    return buf, buf[:k], buf[k:].view(torch.int32)


def topk_compress(x, k):
    x = dev_f32(x)
    n = x.numel()
    buf, vals, idx = new_payload(k, x.device)
    ws = topk_workspace(n, k, x.device)
    _lib.call("grace_topk_compress", _p(x), n, k, _p(vals), _p(idx), _p(ws), ws.numel(), _stream())
    return buf, vals, idx


def topk_residual_step(g, residual, has_residual, beta, gamma, k, out=None, payload=None):
    g = dev_f32(g)
    n = g.numel()
    buf, vals, idx = new_payload(k, g.device) if payload is None else payload
    ws = topk_workspace(n, k, g.device)
    _lib.call("grace_topk_residual_step", _p(g), _p(residual), 1 if has_residual else 0, float(beta),
              float(gamma), n, k, _p(vals), _p(idx), _p(out), _p(ws), ws.numel(), _stream())
    return buf, vals, idx


def topk_status(n, k, device):
    """Whether the last top-k launch on this stream took the exact fallback (syncs; tests only)."""
    import ctypes
    ws = topk_workspace(n, k, device)
    st = ctypes.c_int32(-1)
    _lib.call("grace_read_status", _p(ws), ctypes.addressof(st), _stream())
    return st.value


def sparse_decode(vals, idx, n):
    vals = dev_f32(vals, "values")
    idx = require_dev(idx, "indices")
    out = torch.empty(n, dtype=F32, device=vals.device)
    if idx.dtype == torch.int32:
        _lib.call("grace_sparse_decode", _p(vals), _p(idx), vals.numel(), _p(out), n, _stream())
    elif idx.dtype == torch.int64:
        _lib.call("grace_sparse_decode_i64", _p(vals), _p(idx), vals.numel(), _p(out), n, _stream())
    else:
        raise TypeError(f"indices must be int32 or int64, got {idx.dtype}")
    return out


_tags = {}


def sparse_aggregate(vals_base, idx_base, stride, counts, world, n, divisor):
    """Rank-ordered decode+aggregate of W sparse payloads laid out rank-major with `stride`."""
    dev = vals_base.device
    tags = _tags.get(str(dev))
    if tags is None or tags.numel() < n:
        tags = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        _tags[str(dev)] = tags
    out = torch.empty(n, dtype=F32, device=dev)
    import ctypes
    arr = (ctypes.c_int64 * world)(*[int(c) for c in counts])
    _lib.call("grace_sparse_aggregate", _p(vals_base), _p(idx_base), int(stride), ctypes.addressof(arr),
              int(world), float(divisor), _p(out), _p(tags), n, _stream())
    return out


# ----------------------------------------------------------------------------- timing helpers
def timer_enable(on=True):
    _lib.call("grace_timer_enable", 1 if on else 0)


def timer_collect():
    import ctypes
    ms = ctypes.c_float(0)
    cnt = ctypes.c_int32(0)
    _lib.call("grace_timer_collect", ctypes.addressof(ms), ctypes.addressof(cnt))
    return ms.value, cnt.value


def isclose_f32_ulps(a, b, ulps):
    """|a - b| <= ulps * ulp(b) elementwise (host helper for tests)."""
    a = torch.as_tensor(a, dtype=torch.float32)
    b = torch.as_tensor(b, dtype=torch.float32)
    spacing = torch.abs(torch.nextafter(b, torch.full_like(b, math.inf)) - b)
    return bool(torch.all(torch.abs(a - b) <= ulps * spacing))
