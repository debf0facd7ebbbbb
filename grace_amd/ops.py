"""Tensor-level wrappers over the C ABI.

Every function takes torch tensors that live on the GPU (torch provides device memory and the
current HIP stream only; all arithmetic runs in libgrace_hip.so), validates dtype / contiguity,
allocates outputs and launches on ``torch.cuda.current_stream()``.
"""
import functools
import math
import os

import torch

from . import _lib

F32 = torch.float32


class GraceDeviceError(TypeError):
    """A grace_amd codec was handed a tensor that is not on the GPU."""


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


_current_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream of the current device, as a raw pointer (no Stream object)."""
    if _raw_stream is not None and _current_device is not None:
        return _raw_stream(_current_device())
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


_reuse = {}
_getrefcount = __import__("sys").getrefcount
_storage_uses = torch._C._storage_Use_Count


def _refcount_selftest():
    """Whether this interpreter and torch count references the way the output / residual reuse
    checks assume (only CPython 3.10 / torch 2.10 were exercised).  Replays the exact
    pattern of OutputRecycler.take -- an entry (tensor, storage cdata, storage) popped from a dict
    and unpacked -- for a dropped tensor (must read "unheld": refcount 3, storage uses 2), a held one
    and a held view (both must read "held").  Any other answer turns every reuse path off: the
    callers then allocate and write densely, exactly as without reuse."""
    def unheld(d):
        ent = d.pop("x")
        buf, cdata, _st = ent
        return _getrefcount(buf) == 3 and _storage_uses(cdata) == 2

    def entry():
        t = torch.empty(8)
        st = t.untyped_storage()
        return t, {"x": (t, st._cdata, st)}
    try:
        t, d = entry()
        del t
        dropped = unheld(d)
        t, d = entry()
        held = unheld(d)
        t, d = entry()
        v = t[1:]
        del t
        view = unheld(d)
        del v
        return dropped and not held and not view
    except Exception:
        return False


# every reuse path (reusable_output, OutputRecycler, ResidualMemory.spare_for, ShardedTopK's spare
# residual) is gated on this
REUSE_OK = _refcount_selftest()


_sign_w1 = None


def launch_sign_step_w1(x, out):
    """grace_sign_step_w1 on a contiguous f32 device tensor into `out`: the launch-bound W=1 path."""
    global _sign_w1
    f = _sign_w1
    if f is None:
        f = _sign_w1 = _lib.fn("grace_sign_step_w1")
    st = f(x.data_ptr(), None, out.data_ptr(), x.numel(), _stream())
    if st:
        _lib.check("grace_sign_step_w1", st)


def reusable_output(slot, shape, dtype, device):
    """An output tensor for a per-step codec result, reused across calls when nobody outside this
    cache still holds the previous one and the call runs on the stream it was made on, so reuse is
    stream-ordered behind every earlier use.  "Nobody holds it" needs two checks: the Python object
    (CPython refcount: tuple + local + argument = 3) and its storage, because a view or reshape
    (``out.view(-1)``, ``out[1:]``) is another tensor on the same storage that the object's refcount
    cannot see -- the StorageImpl use count is 2 exactly when only the cached tensor and the cached
    storage handle refer to it.  A caller that keeps its results, or any view of them, gets a fresh
    tensor each call, exactly as the reference's new allocations; one that consumes and drops them
    (``grad.copy_(grc.step(grad, name))``, examples/dist/CIFAR10-dawndist/core.py:204-206) skips
    the allocator on launch-bound steps."""
    key = (slot, shape, dtype, device, _stream())
    hit = _reuse.get(key)
    if hit is not None:
        buf = hit[0]
        if REUSE_OK and _getrefcount(buf) == 3 and _storage_uses(hit[1]) == 2:
            return buf
    buf = torch.empty(shape, dtype=dtype, device=device)
    _reuse[key] = (buf, buf.untyped_storage()._cdata, buf.untyped_storage())
    return buf


class OutputRecycler:
    """Per-name recycled dense outputs of the world-1 top-k step.  A step's result is zero except at
    its payload positions; when the caller has dropped it (no tensor or view of its storage left
    outside this cache: the reusable_output test) and never modified it (the tensor version counter
    that views share is unchanged), the next step of the same name on the same stream gets it back
    together with the payload indices, and the kernels zero those positions and write only their
    own selection instead of rewriting all n elements (grace_topk_residual_step_carry, prev_idx).
    A caller that keeps or edits its results gets a fresh tensor and the dense write, as before."""

    def __init__(self):
        self._hit = {}
        self.hits = 0      # steps that got their previous result back (sparse write)
        self.dense_hits = 0   # steps that got it back to rewrite densely (take(dense=True))
        self.misses = 0    # steps that allocated (first step, result held / edited, other stream)

    def take(self, name, like, alloc=True, dense=False):
        """(out tensor, prev_idx or None) for the next step of `name` shaped like `like` (a tensor, or
        a (numel, device) pair for an f32 vector).  A miss allocates (torch.empty_like) unless
        alloc=False, which returns (None, None) and leaves the allocation to the caller.  dense=True:
        the caller rewrites every element (the buffer is kept for its placement, not to skip
        writes); such hits are counted in dense_hits."""
        numel, device = (like.numel(), like.device) if isinstance(like, torch.Tensor) else (int(like[0]), like[1])
        hit = self._hit.pop(name, None)
        if hit is not None:
            buf, cdata, storage, version, prev_idx, key = hit
            # references to buf: the popped tuple, the local name, getrefcount's argument
            if (REUSE_OK and key == (numel, torch.device(device), _stream()) and _getrefcount(buf) == 3
                    and _storage_uses(cdata) == 2 and buf._version == version):
                if dense:
                    self.dense_hits += 1
                else:
                    self.hits += 1
                return buf, prev_idx
        self.misses += 1
        if not alloc:
            return None, None
        if isinstance(like, torch.Tensor):
            return torch.empty_like(like), None
        return torch.empty(numel, dtype=F32, device=device), None

    def keep(self, name, out, idx):
        """Remember this step's result and its payload indices (int32, length k)."""
        st = out.untyped_storage()
        self._hit[name] = (out, st._cdata, st, out._version, idx, (out.numel(), out.device, _stream()))

    def drop(self, name):
        """Forget `name`'s previous result (its next step allocates and writes densely)."""
        self._hit.pop(name, None)

    def clear(self):
        self._hit.clear()


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
def _out_buf(out, n, dtype, device, what):
    """a caller-provided output (a view into a send record) or a new tensor"""
    if out is None:
        return torch.empty(n, dtype=dtype, device=device)
    if out.dtype != dtype or out.numel() != n or not out.is_contiguous() or out.device != device:
        raise ValueError(f"{what}: out must be a contiguous {dtype} tensor of {n} elements on {device}")
    return out


def sign_encode(x, out=None):
    x = dev_f32(x)
    codes = _out_buf(out, x.numel(), torch.uint8, x.device, "sign_encode")
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


def sign_step_w1(x, want_codes=True, reuse_out=False):
    if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == F32 and x.is_contiguous()):
        x = dev_f32(x)   # (the checks dev_f32 would make, without its reshape on the common path)
    codes = torch.empty(x.numel(), dtype=torch.uint8, device=x.device) if want_codes else None
    out = reusable_output("sign_w1", x.shape, F32, x.device) if reuse_out else torch.empty_like(x)
    _lib.call("grace_sign_step_w1", x.data_ptr(), _p(codes), out.data_ptr(), x.numel(), _stream())
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
TOPK_SMALL_N = 32768   # topk.hip kSmallN: buckets up to this size run in one workgroup (dense writes)


def ratio_k(numel, ratio):
    """k = max(1, int(numel * ratio)) (grace_dl/dist/compressor/topk.py:34)."""
    return max(1, int(numel * ratio))


class TopKWaitError(_lib.GraceNativeError):
    """A wait of the top-k parallel exact fallback ran out in an earlier call (status bit 2 of the
    registered pinned word, include/grace_hip.h grace_topk_status_word): that call's payload,
    residual and output are not valid.  Never expected: the fallback's waits are only on slices that
    running workgroups have claimed (csrc/topk.hip parallel_exact)."""


_tk_st = None


def _topk_status():
    """The pinned word every top-k launch of this process reports a fallback run-out to (registered
    once), checked at every top-k call: it covers the earlier calls whose kernels have finished."""
    global _tk_st
    hit = _tk_st
    if hit is None:
        st = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        _lib.call("grace_topk_status_word", st.data_ptr())
        hit = _tk_st = (st, st.numpy())     # numpy view: a plain host read per call
    if hit[1][0]:
        v = int(_lib.query("grace_status_take", hit[0].data_ptr()))   # read-and-clear, host atomic
        if v & 2:
            raise TopKWaitError("grace_amd: a top-k exact-fallback wait ran out in an earlier call; its "
                                "payload, residual and output were not valid -- discard the residual / "
                                "sharded state of the names stepped since the last check (e.g. "
                                "memory.residuals.pop(name)), or run with TopKCompressor(check_sync=True) "
                                "so the failing step itself raises")
    return hit[0]


def topk_check():
    """Wait for the device, then raise TopKWaitError if any top-k launch so far aborted
    (TopKCompressor(check_sync=True) calls this after every step)."""
    torch.cuda.synchronize()
    _topk_status()


def topk_fallback_spin_limit(limit=-1):
    """Bound of each parallel exact-fallback wait in microseconds of device wall time (default
    2 s, so only a true hang trips it; tests force 0); returns the previous bound."""
    return int(_lib.query("grace_topk_fallback_spin_limit", int(limit)))


def topk_workspace(n, k, device):
    _topk_status()
    return workspace("topk", _lib.query("grace_topk_workspace_bytes", n, k), device)


# Buffer placement (r06): on MI355X the fused step's main pass (g, r read; r', out
# written) runs at 171-174 us or at 184-193 us on a 256 MiB bucket depending on WHICH pair of
# allocations holds r and out -- a property of the pair, not of offsets inside them
# (profiles/r06_place4_5.txt).  At a large bucket's first step, pick_pair tries a few residual and
# output allocations against the step's gradient with the pass's own streaming skeleton
# (grace_topk_stream_probe) and keeps the fastest pair; the output buffer then stays with the name
# (the dropped previous result comes back and is rewritten densely).  One host synchronisation per
# name; GRACE_PLACE_PROBE=0 turns it off.
PLACE_PROBE = os.environ.get("GRACE_PLACE_PROBE", "1") != "0"
PLACE_MIN_N = 1 << 24
# the residual candidates' positions, in GiB of allocations from the first (in twos, spread out)
PLACE_RES_GIB = tuple(float(x) for x in os.environ.get("GRACE_PLACE_RES_GIB", "0,0,4,4,12,12").split(","))
PLACE_RES = len(PLACE_RES_GIB)
# the output candidates' distances past the residual candidates, in GiB of allocations: on one GPU
# fitting pairs were 1-6 GiB apart, on another only >= 8 GiB (profiles/r06_spacer.txt)
PLACE_OUT_GIB = tuple(float(x) for x in os.environ.get("GRACE_PLACE_OUT_GIB", "0,3,8,16,32").split(","))
PLACE_OUT = len(PLACE_OUT_GIB)


def _spacer(gib, held):
    """gib GiB of device memory straight from the runtime (grace_spacer_alloc), kept in `held`."""
    import ctypes
    p = ctypes.c_void_p()
    _lib.call("grace_spacer_alloc", int(gib * (1 << 30)), ctypes.addressof(p))
    held.append(p.value)


def pick_pair(g, res_gib=None, out_gib=None):
    """(residual, output, probe microseconds per pair): the fastest of n_res x len(out_gib) fresh
    allocation pairs under the stream probe over g (their contents are garbage: the caller's first
    step writes both densely).  The residual candidates are allocated res_gib GiB of allocations
    past the first one, the output candidates out_gib GiB past the last residual candidate; the
    spacers between are plain runtime allocations (grace_spacer_alloc), given back as soon as the
    candidates are placed."""
    res_gib = PLACE_RES_GIB if res_gib is None else tuple(res_gib)
    out_gib = PLACE_OUT_GIB if out_gib is None else tuple(out_gib)
    g = dev_f32(g)
    n = g.numel()
    n_res, n_out = len(res_gib), len(out_gib)
    spacer_gib = max(res_gib) + max(out_gib)
    need = 4 * n * (n_res + n_out) + int(spacer_gib * (1 << 30))
    if torch.cuda.mem_get_info(g.device)[0] < need + (4 << 30):
        return torch.empty_like(g), torch.empty_like(g), []
    ws = workspace("probe", _lib.query("grace_topk_stream_probe_workspace_bytes", n), g.device)
    held, rs, outs = [], [], []
    try:
        done = 0.0
        for gib in sorted(res_gib):
            if gib - done > 0:
                _spacer(gib - done, held)
            done = gib
            rs.append(torch.empty_like(g))
        done = 0.0
        for gib in sorted(out_gib):
            if gib - done > 0:
                _spacer(gib - done, held)
            done = gib
            outs.append(torch.empty_like(g))
    except (torch.cuda.OutOfMemoryError, _lib.GraceNativeError):
        rs = outs = None
        return torch.empty_like(g), torch.empty_like(g), []
    finally:
        for q in held:
            _lib.call("grace_spacer_free", q)
    pairs = [(i, j) for j in range(n_out) for i in range(n_res)]
    evs = []
    for i, j in pairs:
        for rep in range(2):   # the second launch is timed (first-touch costs out of the figure)
            if rep == 1:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            _lib.call("grace_topk_stream_probe", _p(g), _p(rs[i]), _p(outs[j]), n, 0, _p(ws), ws.numel(), _stream())
        e1.record()
        evs.append((e0, e1))
    evs[-1][1].synchronize()
    us = [a.elapsed_time(b) * 1e3 for a, b in evs]
    best = min(range(len(pairs)), key=lambda q: us[q])
    i, j = pairs[best]
    return rs[i], outs[j], us


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


def topk_step_dense(x, k, out=None, prev_idx=None):
    """World-1 Allgather(TopK, NoneMemory).step in one streaming pass (grace_topk_step_dense): the
    payload of topk_compress plus the dense (0 + decode) / 1 result; x is only read.  prev_idx: the
    payload indices of the earlier step whose result `out` still holds unmodified (recycled)."""
    x = dev_f32(x)
    n = x.numel()
    buf, vals, idx = new_payload(k, x.device)
    out = torch.empty(n, dtype=F32, device=x.device) if out is None else out
    ws = topk_workspace(n, k, x.device)
    _lib.call("grace_topk_step_dense", _p(x), n, k, _p(vals), _p(idx), _p(out), _p(prev_idx),
              prev_idx.numel() if prev_idx is not None else 0, _p(ws), ws.numel(), _stream())
    return buf, vals, idx, out


def topk_residual_step(g, residual, has_residual, beta, gamma, k, out=None, payload=None, carry=None,
                       carry_valid=False, prev_idx=None):
    """carry: f32[topk_carry_size(n, k)] kept with `residual` (grace_topk_residual_step_carry);
    carry_valid: it holds the samples the previous step of this residual wrote.  prev_idx: int32
    payload indices of the earlier step whose result `out` still holds unmodified (a recycled
    output: the step zeroes those and writes only its own selection)."""
    g = dev_f32(g)
    n = g.numel()
    buf, vals, idx = new_payload(k, g.device) if payload is None else payload
    ws = topk_workspace(n, k, g.device)
    if carry is not None and (carry.dtype != F32 or not carry.is_contiguous()):
        raise ValueError("grace_amd: the top-k carry is a contiguous float32 device tensor")
    if prev_idx is not None and (out is None or prev_idx.dtype != torch.int32 or not prev_idx.is_contiguous()):
        raise ValueError("grace_amd: prev_idx needs an output and contiguous int32 indices")
    if carry is None and prev_idx is None:
        _lib.call("grace_topk_residual_step", _p(g), _p(residual), 1 if has_residual else 0, float(beta),
                  float(gamma), n, k, _p(vals), _p(idx), _p(out), _p(ws), ws.numel(), _stream())
    else:
        _lib.call("grace_topk_residual_step_carry", _p(g), _p(residual), 1 if has_residual else 0, float(beta),
                  float(gamma), n, k, _p(vals), _p(idx), _p(out), _p(carry), carry.numel() if carry is not None else 0,
                  1 if carry_valid else 0, _p(prev_idx), prev_idx.numel() if prev_idx is not None else 0,
                  _p(ws), ws.numel(), _stream())
    return buf, vals, idx


def topk_residual_step_swap(g, residual, has_residual, beta, gamma, k, residual_out, payload=None, carry=None,
                            carry_valid=False):
    """The world > 1 residual step into a second residual buffer (grace_topk_residual_step_swap):
    reads g and `residual`, writes `residual_out` (distinct) and the payload."""
    g = dev_f32(g)
    n = g.numel()
    buf, vals, idx = new_payload(k, g.device) if payload is None else payload
    ws = topk_workspace(n, k, g.device)
    if residual_out is None or residual_out.data_ptr() == (residual.data_ptr() if residual is not None else 0):
        raise ValueError("grace_amd: topk_residual_step_swap needs a distinct residual_out")
    _lib.call("grace_topk_residual_step_swap", _p(g), _p(residual) if has_residual else None, 1 if has_residual else 0,
              float(beta), float(gamma), n, k, _p(vals), _p(idx), _p(residual_out), _p(carry),
              carry.numel() if carry is not None else 0, 1 if carry_valid else 0, _p(ws), ws.numel(), _stream())
    return buf, vals, idx


@functools.lru_cache(maxsize=256)
def topk_carry_size(n, k):
    """Length of the residual-sample carry for an (n, k) step, 0 where the step has none."""
    return int(_lib.query("grace_topk_carry_size", n, k))


class MainEvent:
    """A native event that completes with the main pass of the next top-k step it is armed for
    (grace_topk_arm_main_event): the next bucket's step on another stream waits on it, so its
    bracket runs beside this bucket's finalize (tools/exp_two_streams.py)."""

    def __init__(self):
        import ctypes
        h = ctypes.c_void_p()
        _lib.call("grace_event_create", ctypes.addressof(h))
        self.handle = h.value

    def arm(self):
        _lib.call("grace_topk_arm_main_event", self.handle)

    def wait(self, stream=None):
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _lib.call("grace_stream_wait_event", s, self.handle)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.call("grace_event_destroy", h)
            except Exception:
                pass


def topk_status(n, k, device):
    """Whether the last top-k launch on this stream took the exact fallback: 0 no, 1 yes, 2 it
    aborted after a wait ran out (syncs; tests only)."""
    import ctypes
    ws = workspace("topk", _lib.query("grace_topk_workspace_bytes", n, k), device)
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


def _agg_tags(dev, n):
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)   # per stream, like workspace()
    tags = _tags.get(key)
    if tags is None or tags.numel() < n:
        tags = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        _tags[key] = tags
    return tags


def sparse_aggregate(vals_base, idx_base, stride, counts, world, n, divisor, out=None):
    """Rank-ordered decode+aggregate of W sparse payloads laid out rank-major with `stride`.
    With `out` given it must already be zero-filled (e.g. by a fill that overlapped the gather)."""
    dev = vals_base.device
    tags = _agg_tags(dev, n)
    prefilled = out is not None
    if out is None:
        out = torch.empty(n, dtype=F32, device=dev)
    import ctypes
    arr = (ctypes.c_int64 * world)(*[int(c) for c in counts])
    _lib.call("grace_sparse_aggregate_into" if prefilled else "grace_sparse_aggregate", _p(vals_base), _p(idx_base),
              int(stride), ctypes.addressof(arr), int(world), float(divisor), _p(out), _p(tags), n, _stream())
    return out


def exchange_record_words(cap):
    return int(_lib.query("grace_exchange_record_words", int(cap)))


def sparse_aggregate_capped(recs, cap, world, n, divisor, stat):
    """Rank-ordered decode+aggregate of W gathered capacity-bounded records (counts read from the
    record headers on the device); stat (int32[2] on the device) <- {max count, overflow flag}."""
    require_dev(recs, "records")
    stride = exchange_record_words(cap)
    if recs.numel() != world * stride or recs.dtype != torch.int32 or stat.numel() < 2:
        raise ValueError("sparse_aggregate_capped: records / stat do not match (world, cap)")
    out = torch.empty(n, dtype=F32, device=recs.device)
    _lib.call("grace_sparse_aggregate_capped", _p(recs), stride, int(cap), int(world), float(divisor), _p(out),
              _p(_agg_tags(recs.device, n)), int(n), _p(stat), _stream())
    return out


SORT_PAYLOAD_MAX_N = 1 << 28   # payload.hip kMaxGroupChunks * chunk: largest bucket sort_payload groups


def _off_words(k):
    return (int(k) + 1) // 2     # u16 chunk offsets of k entries, in 4-B words


def sorted_payload_len(k, n):
    """4-B words of a chunk-grouped payload: [vals f32[k] | offsets u16[k] (padded to a word) |
    chunk ends u32[ceil(n/8192)]] -- 6 B per entry on the wire instead of the packed payload's 8."""
    return int(k) + _off_words(k) + (int(n) + 8191) // 8192


def sort_payload(buf, k, n):
    """Packed payload [vals f32[k] | idx i32[k]] -> a new chunk-grouped payload
    [vals | u16 offsets inside the chunk | chunk end offsets] (sorted_payload_len(k, n) words)."""
    out = torch.empty(sorted_payload_len(k, n), dtype=F32, device=buf.device)
    ws = workspace("sortpay", _lib.query("grace_sort_payload_workspace_bytes", k, n), buf.device)
    _lib.call("grace_sort_payload", _p(buf), _p(buf[k:]), int(k), int(n), _p(out), _p(out[k:]),
              _p(out[k + _off_words(k):]), _p(ws), ws.numel(), _stream())
    return out


def sparse_aggregate_sorted(gathered, k, world, n, divisor):
    """Rank-ordered aggregate of W chunk-grouped payloads (rank-major, stride sorted_payload_len)."""
    out = torch.empty(n, dtype=F32, device=gathered.device)
    stride = sorted_payload_len(k, n)
    _lib.call("grace_sparse_aggregate_sorted", _p(gathered), _p(gathered[k:]), _p(gathered[k + _off_words(k):]),
              stride, int(world), float(divisor), _p(out), int(n), _stream())
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


# ----------------------------------------------------------------------------- segmented tables
_seg_cache = {}


def seg_tables(sizes, unit, device):
    """Device offset tables for a segmented bucket: (seg_off[nseg+1], sub_off[nseg+1], nsub) where
    sub_off counts ceil(n_s / unit) sub-blocks (QSGD buckets, TernGrad work units) per segment.
    Cached: built (one small H2D copy) once per shape."""
    key = (tuple(int(s) for s in sizes), int(unit), str(device))
    hit = _seg_cache.get(key)
    if hit is None:
        seg = [0]
        sub = [0]
        for s in key[0]:
            seg.append(seg[-1] + s)
            sub.append(sub[-1] + (s + unit - 1) // unit)
        hit = (torch.tensor(seg, dtype=torch.int64).to(device), torch.tensor(sub, dtype=torch.int64).to(device),
               sub[-1])
        _seg_cache[key] = hit
    return hit


def _opt(t):
    return t.data_ptr() if t is not None else None


# ----------------------------------------------------------------------------- QSGD
def qsgd_compress(x, quantum_num, bucket_size, sizes=None, variant=0, u=None, seed=0, norms_in=None, xoff=0,
                  codes_out=None, norms_out=None):
    """x: flat f32 device buffer (one tensor, or `sizes` segments back to back).  xoff: the element
    of a larger bucket x[0] is (a shard starting on a bucket boundary): the device generator draws
    by that bucket's element index (grace_qsgd_compress_at).  codes_out / norms_out: write there
    (views into a send record) instead of new tensors."""
    x = dev_f32(x)
    sizes = [x.numel()] if sizes is None else sizes
    seg_off, bkt_off, nb = seg_tables(sizes, bucket_size, x.device)
    codes = _out_buf(codes_out, x.numel(), torch.int8 if quantum_num < 128 else torch.float16, x.device,
                     "qsgd_compress")
    norms = _out_buf(norms_out, nb, F32, x.device, "qsgd_compress norms")
    _lib.call("grace_qsgd_compress_at", _p(x), int(xoff), _p(seg_off), _p(bkt_off), len(sizes), nb, int(quantum_num),
              int(bucket_size), int(variant), _opt(u), int(seed) & (2 ** 64 - 1), _opt(norms_in), _p(norms),
              _p(codes), _stream())
    return codes, norms


def qsgd_step_w1_ok(sizes, bucket_size):
    return int(bucket_size) == 128 and len(sizes) <= _lib.query("grace_qsgd_seg_max")


def qsgd_step_w1(x, quantum_num, sizes=None, variant=0, u=None, seed=0):
    """World-1 Allgather(QSGD(q, bucket 128)).step in one pass (grace_qsgd_step_w1): the codes of
    qsgd_compress decoded as (0 + d) / 1 without being stored; `sizes` segments as qsgd_compress."""
    x = dev_f32(x)
    sizes = [x.numel()] if sizes is None else sizes
    seg_off, bkt_off, nb = seg_tables(sizes, 128, x.device)
    out = torch.empty(x.numel(), dtype=F32, device=x.device)
    _lib.call("grace_qsgd_step_w1", _p(x), _p(seg_off), _p(bkt_off), len(sizes), nb, int(quantum_num), int(variant),
              _opt(u), int(seed) & (2 ** 64 - 1), _p(out), _stream())
    return out


def qsgd_decompress(codes, norms, quantum_num, bucket_size, n, sizes=None, variant=0, world=1,
                    aggregate=False, divisor=1.0):
    codes, norms = require_dev(codes), require_dev(norms)
    sizes = [n] if sizes is None else sizes
    seg_off, bkt_off, nb = seg_tables(sizes, bucket_size, codes.device)
    out = torch.empty(n, dtype=F32, device=codes.device)
    _lib.call("grace_qsgd_decompress", _p(codes), _p(norms), n, nb, int(world), _p(seg_off), _p(bkt_off),
              len(sizes), n, int(quantum_num), int(bucket_size), int(variant), 1 if aggregate else 0,
              float(divisor), _p(out), _stream())
    return out


def qsgd_decompress_records(records, rec_bytes, norm_off, world, units_per_rank, rank_lo, quantum_num, n, sizes=None,
                            variant=0):
    """Sharded QSGD's replicated decode (bucket 128) straight from the W gathered per-rank records
    (grace_qsgd_decompress_records): rank w's codes from byte w * rec_bytes, its bucket norms from
    byte w * rec_bytes + norm_off; rank_lo: device int64[W], each rank's first element."""
    records = require_dev(records)
    sizes = [n] if sizes is None else sizes
    seg_off, bkt_off, _ = seg_tables(sizes, 128, records.device)
    out = torch.empty(n, dtype=F32, device=records.device)
    _lib.call("grace_qsgd_decompress_records", _p(records), int(rec_bytes), int(norm_off), int(world),
              int(units_per_rank), _p(rank_lo), _p(seg_off), _p(bkt_off), len(sizes), int(n), int(quantum_num),
              int(variant), _p(out), _stream())
    return out


def qsgd_global_compress(x, quantum_num, u=None, seed=0, norm_in=None):
    """Horovod-flavour QSGD (grace_dl/torch/compressor/qsgd.py:12-31): one norm over the tensor.
    Returns (codes int8 | fp16 [n], norm f32[1])."""
    x = dev_f32(x)
    n = x.numel()
    codes = torch.empty(n, dtype=torch.int8 if quantum_num < 128 else torch.float16, device=x.device)
    norm = torch.empty(1, dtype=F32, device=x.device)
    ws = workspace("qsgd_global", _lib.query("grace_qsgd_global_workspace_bytes"), x.device)
    _lib.call("grace_qsgd_global_compress", _p(x), n, int(quantum_num), _opt(u), int(seed) & (2 ** 64 - 1),
              _opt(norm_in), _p(norm), _p(codes), _p(ws), _stream())
    return codes, norm


def qsgd_global_decompress(codes, norm, quantum_num, n, world=1, aggregate=False, divisor=1.0):
    """(norm / q) * code (qsgd.py:33-38): the bucketed decoder with one bucket of n elements."""
    return qsgd_decompress(codes, norm, quantum_num, n, n, world=world, aggregate=aggregate, divisor=divisor)


# ----------------------------------------------------------------------------- TernGrad
def terngrad_compress(x, sizes=None, clip=None, u=None, seed=0):
    x = dev_f32(x)
    sizes = [x.numel()] if sizes is None else sizes
    unit = _lib.query("grace_terngrad_unit")
    seg_off, unit_off, nunits = seg_tables(sizes, unit, x.device)
    codes = torch.empty(x.numel(), dtype=torch.int8, device=x.device)
    scalars = torch.empty(len(sizes), dtype=F32, device=x.device)
    ws = workspace("terngrad", _lib.query("grace_terngrad_workspace_bytes", nunits), x.device)
    _lib.call("grace_terngrad_compress", _p(x), _p(seg_off), _p(unit_off), len(sizes), nunits, _opt(clip),
              _opt(u), int(seed) & (2 ** 64 - 1), _p(codes), _p(scalars), _p(ws), _stream())
    return codes, scalars


def terngrad_step_w1(x, sizes=None, clip=None, u=None, seed=0):
    """World-1 Allgather(TernGrad).step (grace_terngrad_step_w1): the statistics pass, then one pass
    writing 0 + code * scalar for the codes terngrad_compress would draw, never storing them."""
    x = dev_f32(x)
    sizes = [x.numel()] if sizes is None else sizes
    unit = _lib.query("grace_terngrad_unit")
    seg_off, unit_off, nunits = seg_tables(sizes, unit, x.device)
    scalars = torch.empty(len(sizes), dtype=F32, device=x.device)
    out = torch.empty(x.numel(), dtype=F32, device=x.device)
    ws = workspace("terngrad", _lib.query("grace_terngrad_workspace_bytes", nunits), x.device)
    _lib.call("grace_terngrad_step_w1", _p(x), _p(seg_off), _p(unit_off), len(sizes), nunits, _opt(clip),
              _opt(u), int(seed) & (2 ** 64 - 1), _p(scalars), _p(ws), _p(out), _stream())
    return out


def terngrad_decompress_records(records, rec_bytes, world, rank_lo, packed, scalars, n, sizes=None):
    """Sharded TernGrad's replicated decode straight from the W gathered per-rank records
    (grace_terngrad_decompress_records): int8 codes, or 2-bit planar packed (packed=True);
    rank_lo: device int64[W + 1], each rank's element range boundaries."""
    records, scalars = require_dev(records), require_dev(scalars)
    sizes = [n] if sizes is None else sizes
    unit = _lib.query("grace_terngrad_unit")
    seg_off, _, _ = seg_tables(sizes, unit, records.device)
    out = torch.empty(n, dtype=F32, device=records.device)
    _lib.call("grace_terngrad_decompress_records", _p(records), int(rec_bytes), int(world), _p(rank_lo),
              1 if packed else 0, _p(scalars), _p(seg_off), len(sizes), int(n), _p(out), _stream())
    return out


def terngrad_decompress(codes, scalars, n, sizes=None, world=1, aggregate=False, divisor=1.0):
    codes, scalars = require_dev(codes), require_dev(scalars)
    sizes = [n] if sizes is None else sizes
    unit = _lib.query("grace_terngrad_unit")
    seg_off, _, _ = seg_tables(sizes, unit, codes.device)
    out = torch.empty(n, dtype=F32, device=codes.device)
    _lib.call("grace_terngrad_decompress", _p(codes), _p(scalars), n, len(sizes), int(world), _p(seg_off),
              len(sizes), n, 1 if aggregate else 0, float(divisor), _p(out), _stream())
    return out


# ----------------------------------------------------------------------------- natural / fp16
def natural_compress(x, rand_int=None, seed=0, xoff=0, out=None):
    """xoff (a multiple of 4): the element of a larger bucket x[0] is, for the device generator."""
    x = dev_f32(x)
    codes = _out_buf(out, x.numel(), torch.uint8, x.device, "natural_compress")
    _lib.call("grace_natural_compress_at", _p(x), int(xoff), x.numel(), _opt(rand_int), int(seed) & (2 ** 64 - 1),
              _p(codes), _stream())
    return codes


def cnat_compress(x, rand=None, deterministic=False, seed=0, xoff=0, out=None):
    """xoff (a multiple of 4): the element of a larger bucket x[0] is, for the device generator."""
    x = dev_f32(x)
    codes = _out_buf(out, x.numel(), torch.uint8, x.device, "cnat_compress")
    _lib.call("grace_cnat_compress_at", _p(x), int(xoff), x.numel(), _opt(rand), 1 if deterministic else 0,
              int(seed) & (2 ** 64 - 1), _p(codes), _stream())
    return codes


def natural_decompress(codes, n, flavour, world=1, aggregate=False, divisor=1.0):
    codes = require_dev(codes)
    out = torch.empty(n, dtype=F32, device=codes.device)
    _lib.call("grace_natural_decompress", _p(codes), n, int(world), n, int(flavour), 1 if aggregate else 0,
              float(divisor), _p(out), _stream())
    return out


def fp16_compress(x, out=None):
    x = dev_f32(x)
    h = _out_buf(out, x.numel(), torch.float16, x.device, "fp16_compress")
    _lib.call("grace_fp16_compress", _p(x), _p(h), x.numel(), _stream())
    return h


def fp16_decompress(h):
    h = require_dev(h)
    out = torch.empty(h.numel(), dtype=F32, device=h.device)
    _lib.call("grace_fp16_decompress", _p(h), _p(out), h.numel(), _stream())
    return out


def w1_elementwise_ok(communicator, tensor):
    """Whether a world-1 Allgather(NoneMemory) step may run as one fused element-wise pass:
    a contiguous 16-B aligned f32 device tensor (anything else takes the unfused path)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.memory.none import NoneMemory
    return (communicator.__class__ is Allgather and communicator.memory.__class__ is NoneMemory
            and int(communicator.world_size) == 1 and isinstance(tensor, torch.Tensor) and tensor.is_cuda
            and tensor.dtype == F32 and tensor.is_contiguous() and tensor.data_ptr() % 16 == 0)


def cast_step_w1(x, mode, seed):
    """grace_cast_step_w1: out = 0 + decompress(compress(x)) for natural (0), cnat (1), cnat
    deterministic (2) or fp16 (3), in one pass; same shape as x."""
    out = torch.empty_like(x)
    _lib.call("grace_cast_step_w1", _p(x), x.numel(), int(mode), int(seed) & (2 ** 64 - 1), _p(out), _stream())
    return out


def fp16_decompress_aggregate(h_all, n, world, divisor=1.0):
    """Allgather-step decode of `world` rank-major f16 payloads of n elements each:
    ((0 + d_0) + ... + d_{W-1}) / divisor in one pass (no division when divisor == 1)."""
    h_all = require_dev(h_all)
    out = torch.empty(n, dtype=F32, device=h_all.device)
    _lib.call("grace_fp16_decompress_aggregate", _p(h_all), int(n), int(world), int(n), float(divisor), _p(out),
              _stream())
    return out


# ----------------------------------------------------------------------------- seeds
def step_seed(*parts):
    """Deterministic 64-bit seed for the device generator from (rank, name, step, ...)."""
    import hashlib
    h = hashlib.blake2b(repr(parts).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little")


def rank_of_process():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


# ----------------------------------------------------------------------------- random-k / threshold
def randomk_indices(seed, numel, k, device):
    idx = torch.empty(k, dtype=torch.int64, device=device)
    _lib.call("grace_randomk_indices", int(seed) & (2 ** 64 - 1), int(numel), int(k), _p(idx), _stream())
    return idx


def randomk_perm_indices(seed, numel, k, device):
    """k distinct indices of [0, numel) (Horovod-flavour randperm(numel)[:k] semantics)."""
    idx = torch.empty(k, dtype=torch.int64, device=device)
    _lib.call("grace_randomk_perm_indices", int(seed) & (2 ** 64 - 1), int(numel), int(k), _p(idx), _stream())
    return idx


def widen_i32(idx32):
    idx32 = require_dev(idx32, "indices")
    out = torch.empty(idx32.numel(), dtype=torch.int64, device=idx32.device)
    _lib.call("grace_widen_i32", _p(idx32), idx32.numel(), _p(out), _stream())
    return out


def randomk_step_w1(g, residual, has_residual, beta, gamma, idx):
    """World-1 Allgather(RandomK, ResidualMemory).step (grace_randomk_step_w1): returns (vals, out)."""
    g = dev_f32(g)
    idx = require_dev(idx, "indices")
    vals = torch.empty(idx.numel(), dtype=F32, device=g.device)
    out = torch.empty_like(g)
    _lib.call("grace_randomk_step_w1", _p(g), _p(residual), 1 if has_residual else 0, float(beta), float(gamma),
              g.numel(), _p(idx), idx.numel(), _p(vals), _p(out), _stream())
    return vals, out


def randomk_shard_step(g, residual, has_residual, beta, gamma, lo, idx, out=None):
    """Sharded random-k (grace_randomk_shard_step): this rank's shard g (global elements
    [lo, lo + g.numel())), the global indices idx; returns vals (t where this rank holds the index,
    +0 elsewhere).  residual updated in place; out (optional): this rank's slice of the result."""
    g = dev_f32(g)
    idx = require_dev(idx, "indices")
    vals = torch.empty(idx.numel(), dtype=F32, device=g.device)
    _lib.call("grace_randomk_shard_step", _p(g), _p(residual), 1 if has_residual else 0, float(beta), float(gamma),
              int(lo), g.numel(), _p(idx), idx.numel(), _p(vals), _p(out), _stream())
    return vals


def randomk_decode(vals, idx, n):
    """zeros(n) with 0 + vals[j] at idx[j] (grace_randomk_decode): the world-1 step's result."""
    vals, idx = require_dev(vals), require_dev(idx, "indices")
    out = torch.empty(int(n), dtype=F32, device=vals.device)
    _lib.call("grace_randomk_decode", _p(vals), _p(idx), idx.numel(), _p(out), int(n), _stream())
    return out


def randomk_step_w1_dense(g, residual, has_residual, beta, gamma, idx, out=None, grp=None, prev_grp=None):
    """The world-1 step's out (and r' in `residual`) in one streaming pass after grouping the indices
    by chunk (grace_randomk_step_w1_dense); no payload.  grp: a per-name uint8 buffer of
    randomk_group_bytes(n, k) receiving this step's grouping; prev_grp: the grouping of the earlier
    step whose result `out` still holds unmodified (recycled output: only its non-zeros are
    cleared and only the drawn positions written)."""
    g = dev_f32(g)
    idx = require_dev(idx, "indices")
    if idx.dtype != torch.int64:
        raise ValueError("grace_amd: random-k indices are int64")
    if prev_grp is not None and (out is None or grp is None):
        raise ValueError("grace_amd: a recycled random-k output needs `out` and this step's `grp`")
    out = torch.empty_like(g) if out is None else out
    n, k = g.numel(), idx.numel()
    ws = workspace("randomk_w1", _lib.query("grace_randomk_step_w1_dense_workspace_bytes", n, k), g.device)
    _lib.call("grace_randomk_step_w1_dense", _p(g), _p(residual), 1 if has_residual else 0, float(beta),
              float(gamma), n, _p(idx), k, _p(out), _p(grp), _p(prev_grp), _p(ws), ws.numel(), _stream())
    return out


def randomk_group_bytes(n, k):
    return int(_lib.query("grace_randomk_group_bytes", int(n), int(k)))


def gather(x, idx):
    x = dev_f32(x)
    idx = require_dev(idx)
    vals = torch.empty(idx.numel(), dtype=F32, device=x.device)
    _lib.call("grace_gather", _p(x), _p(idx), idx.numel(), _p(vals), _stream())
    return vals


def threshold_compress(x, thr):
    """(vals f32[m], idx int32[m]) with m data-dependent: one host sync to size the outputs."""
    import numpy as np
    x = dev_f32(x)
    n = x.numel()
    ws = workspace("threshold", _lib.query("grace_threshold_workspace_bytes", n), x.device)
    thr32 = float(np.float32(thr))
    _lib.call("grace_threshold_count", _p(x), n, thr32, _p(ws), _stream())
    meta = ws[:12].view(torch.int32).cpu()
    if int(meta[2]) != 0:
        bound = float(meta[0:1].view(torch.float32)[0])
        _lib.call("grace_threshold_recount", _p(x), n, bound, _p(ws), _stream())
        meta = ws[:12].view(torch.int32).cpu()
    m = int(meta[1])
    vals = torch.empty(m, dtype=F32, device=x.device)
    idx = torch.empty(m, dtype=torch.int32, device=x.device)
    if m:
        _lib.call("grace_threshold_write", _p(x), n, _p(ws), _p(vals), _p(idx), _stream())
    return vals, idx


def threshold_compress_strict(x, thr):
    """Horovod flavour (grace_dl/torch/compressor/threshold.py:17): (vals f32[m], idx int64[m]) of
    |x| > f32(thr) in ascending order; one host sync sizes the outputs."""
    import numpy as np
    x = dev_f32(x)
    n = x.numel()
    t32 = np.float32(thr)
    bound = np.float32("nan") if t32 == np.inf else np.nextafter(t32, np.float32(np.inf))
    ws = workspace("threshold", _lib.query("grace_threshold_workspace_bytes", n), x.device)
    _lib.call("grace_threshold_count_fixed", _p(x), n, float(bound), _p(ws), _stream())
    m = int(ws[:12].view(torch.int32).cpu()[1])
    vals = torch.empty(m, dtype=F32, device=x.device)
    idx = torch.empty(m, dtype=torch.int64, device=x.device)
    if m:
        _lib.call("grace_threshold_write_i64", _p(x), n, _p(ws), _p(vals), _p(idx), _stream())
    return vals, idx


# ----------------------------------------------------------------------------- PowerSGD
def powersgd_p(M2d, q):
    n, m = M2d.shape
    r = q.shape[1]
    P = torch.empty(n, r, dtype=F32, device=M2d.device)
    ws = workspace("powersgd", _lib.query("grace_powersgd_workspace_bytes", n, m, r), M2d.device)
    _lib.call("grace_powersgd_p", _p(M2d), n, m, _p(require_dev(q)), r, _p(P), _p(ws), _stream())
    return P


def powersgd_p_draw(M2d, r, seed, out=None):
    """P = M q with q = ops.normal((m, r), seed), drawn inside the contraction (no q buffer);
    out: an n x r f32 view to write P into (a send record)."""
    n, m = M2d.shape
    P = _out_buf(out.reshape(-1) if out is not None else None, n * r, F32, M2d.device, "powersgd_p_draw").view(n, r)
    ws = workspace("powersgd", _lib.query("grace_powersgd_workspace_bytes", n, m, r), M2d.device)
    _lib.call("grace_powersgd_p_draw", _p(M2d), n, m, int(seed) & (2 ** 64 - 1), int(r), _p(P), _p(ws), _stream())
    return P


def powersgd_qt(M2d, P):
    n, m = M2d.shape
    r = P.shape[1]
    Q = torch.empty(m, r, dtype=F32, device=M2d.device)
    ws = workspace("powersgd", _lib.query("grace_powersgd_workspace_bytes", n, m, r), M2d.device)
    _lib.call("grace_powersgd_qt", _p(M2d), n, m, _p(require_dev(P)), r, _p(Q), _p(ws), _stream())
    return Q


def powersgd_w1_ok(M2d, r):
    """Whether the one-pass world-1 compress (grace_powersgd_w1_compress) takes this matrix."""
    n, m = M2d.shape
    return (M2d.is_contiguous() and M2d.data_ptr() % 16 == 0 and
            bool(_lib.query("grace_powersgd_w1_ok", n, m, r)))


def powersgd_w1_compress(M2d, q=None, seed=0):
    """World-size-1 rank-4 compress in one pass over M: (P, Q) with P = orthogonalize(M q) and
    Q = M^T P; q is the given [m x 4] matrix, or drawn from `seed` (the ops.normal stream)."""
    n, m = M2d.shape
    dev = M2d.device
    P = torch.empty(n, 4, dtype=F32, device=dev)
    Q = torch.empty(m, 4, dtype=F32, device=dev)
    ws = workspace("powersgd_w1", _lib.query("grace_powersgd_w1_workspace_bytes", n, m), dev)
    status = _w1_status(dev)
    _w1_order(dev)
    _lib.call("grace_powersgd_w1_compress", _p(M2d), n, m, _p(require_dev(q)) if q is not None else None,
              int(seed) & (2 ** 64 - 1), _p(P), _p(Q), _p(ws), ws.numel(), status.data_ptr(), _stream())
    return P, Q


_w1_last = {}


def _w1_order(dev):
    """The one-pass kernels spin on a grid of one workgroup per CU: two such grids running at once
    (calls on two streams) could each hold CUs the other waits for.  So a call issued on a stream
    other than the previous call's first waits for everything already queued there (an event
    recorded only when the stream changes: no cost for one-stream callers)."""
    key = str(dev)
    cur = torch.cuda.current_stream(dev)
    last = _w1_last.get(key)
    if last is not None and last.cuda_stream != cur.cuda_stream:
        ev = torch.cuda.Event()
        ev.record(last)
        cur.wait_event(ev)
    _w1_last[key] = cur


class PowerSGDWaitError(RuntimeError):
    """A wait of the one-pass PowerSGD kernels ran out in an earlier call: that call's P and Q were
    not valid (grace_powersgd_w1_compress, status bit 1)."""


_w1_st = {}


def _w1_status(dev):
    """The pinned status word the one-pass PowerSGD kernels write (include/grace_hip.h), checked
    here at every call: it covers the earlier calls whose kernels have finished since.  Bit 1 (a
    wait ran out: that call's P and Q were not valid) raises PowerSGDWaitError."""
    key = str(dev)
    hit = _w1_st.get(key)
    if hit is None:
        st = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        hit = _w1_st[key] = (st, st.numpy())     # numpy view: a plain host read per call
    st, view = hit
    if view[0]:
        # read-and-clear as one host atomic exchange: a bit a still-running kernel sets between a
        # plain read and a plain clear would be lost
        v = int(_lib.query("grace_status_take", st.data_ptr()))
        if v & 2:
            raise PowerSGDWaitError("grace_amd: a one-pass PowerSGD wait ran out in an earlier call; its P and Q "
                                    "were not valid (never expected: another kernel kept its workgroups from "
                                    "becoming resident)")
    return st


def powersgd_w1_check():
    """Wait for the device and check the one-pass PowerSGD status word (raises on bit 1)."""
    torch.cuda.synchronize()
    for key in list(_w1_st):
        _w1_status(key)


def orthogonalize_(A):
    """In place: A must be a contiguous (row-major) device matrix, or the result would land on a copy."""
    if not isinstance(A, torch.Tensor) or A.device.type != "cuda":
        raise GraceDeviceError(f"grace_amd: orthogonalize_ needs a GPU tensor; got {getattr(A, 'device', type(A))}")
    if not A.is_contiguous() or A.dtype != F32 or A.dim() != 2:
        raise ValueError("grace_amd: orthogonalize_ works in place on a contiguous 2-D float32 matrix")
    _lib.call("grace_orthogonalize", _p(A), A.shape[0], A.shape[1], _stream())
    return A


def normal_orthogonal(shape, seed, device):
    """orthogonalize(normal draws of `shape`) in one launch (draws as ops.normal)."""
    A = torch.empty(shape, dtype=F32, device=device)
    _lib.call("grace_normal_orthogonal", _p(A), shape[0], shape[1], int(seed) & (2 ** 64 - 1), _stream())
    return A


def powersgd_outer(P, Q, M2d=None, want_out=True, want_residual=False):
    n, r = P.shape
    m = Q.shape[0]
    dev = P.device
    out = torch.empty(n, m, dtype=F32, device=dev) if want_out else None
    res = torch.empty(n, m, dtype=F32, device=dev) if want_residual else None
    _lib.call("grace_powersgd_outer", _p(P), _p(Q), n, m, r, _p(out) if out is not None else None,
              _p(M2d) if M2d is not None else None, _p(res) if res is not None else None, _stream())
    return out, res


def normal(shape, seed, device):
    x = torch.empty(shape, dtype=F32, device=device)
    _lib.call("grace_normal_fill", _p(x), x.numel(), int(seed) & (2 ** 64 - 1), _stream())
    return x


# ----------------------------------------------------------------------------- sharded top-k
def shard_record_words(cap):
    """int32 words of one rank's sharded top-k record: [header | vals f32[cap] | local idx i32[cap]]."""
    return int(_lib.query("grace_shard_record_words", int(cap)))


SHARD_HDR = 8   # shard.hip kShHdr: header words (word 0 = the shard length)


def shard_select(recs, world, rank, cap, tab, k, residual, out, out_base, pay_idx, status, sel_gi=None):
    """grace_shard_select over the W gathered records: the exact global top-k (dense output into the
    zero-filled `out`, which covers global [out_base, out_base + out.numel())), this rank's residual
    restored where the global cut rejects a local pick, pay_idx = global index or -1 per own entry.
    `status`: pinned int32 word (bit 1: a record's shard length differs from the agreed `tab`).
    sel_gi: optional int32[world * cap] <- every entry's global index if selected, else -1."""
    dev = recs.device
    if sel_gi is not None and (sel_gi.dtype != torch.int32 or sel_gi.numel() < int(world) * int(cap)):
        raise ValueError("shard_select: sel_gi must be int32 with world * cap elements")
    ws = workspace("shardsel", _lib.query("grace_shard_select_workspace_bytes", int(world), int(cap)), dev)
    _lib.call("grace_shard_select", _p(recs), int(world), int(rank), int(cap), _p(tab), int(k), _p(residual),
              _p(out), int(out_base), out.numel(), _p(pay_idx), _opt(sel_gi), _p(ws), ws.numel(), status.data_ptr(),
              _stream())


def shard_clear(out, out_base, sel_gi):
    """Zero the positions a previous shard_select wrote (its sel_gi) in a recycled output."""
    _lib.call("grace_shard_clear", _p(out), int(out_base), out.numel(), _p(sel_gi), sel_gi.numel(), _stream())
    return out


def new_status_word():
    """A pinned, device-visible int32 status word that kernels set bits in (system-scope fetch_or)."""
    return torch.zeros(1, dtype=torch.int32, pin_memory=True)


def status_take(st):
    """Bits set in a pinned status word since the last take (host atomic exchange; never blocks)."""
    return int(_lib.query("grace_status_take", st.data_ptr())) if int(st[0]) else 0


# ----------------------------------------------------------------------------- DGC
# the sampled threshold thr0 = torch.topk(sample, ks)[0].min() (dgc.py:20-21) by the three-digit
# radix select (grace_dgc_sample_kth) instead of the sample's full top-k; GRACE_DGC_SAMPLE_KTH=0
# takes the top-k engine's values instead (A/B; the thresholds are identical)
DGC_SAMPLE_KTH = os.environ.get("GRACE_DGC_SAMPLE_KTH", "1") != "0"


def dgc_sample_kth(sample, ks):
    """(1,) f32: the ks-th largest sampled magnitude, NaN if any sample is NaN -- what
    torch.topk(sample, ks)[0].min() gives (grace_dgc_sample_kth)."""
    sample = dev_f32(sample)
    ns = sample.numel()
    if not 1 <= ks <= ns:
        raise ValueError(f"dgc_sample_kth: ks={ks} outside [1, {ns}]")
    out = torch.empty(1, dtype=F32, device=sample.device)
    ws = workspace("dgc_kth", _lib.query("grace_dgc_sample_kth_workspace_bytes"), sample.device)
    _lib.call("grace_dgc_sample_kth", _p(sample), ns, int(ks), _p(ws), _p(out), _stream())
    return out


def _dgc_sample_top(sample, ks):
    """(top values, their count) whose minimum is thr0: the k-th value alone, or the top-k's values"""
    if DGC_SAMPLE_KTH:
        return dgc_sample_kth(sample, ks), 1
    _, top, _ = topk_compress(sample, ks)
    return top, ks


def dgc_compress(t, ratio, sample_idx=None, seed=0):
    """DgcCompressor.compress (dgc.py:12-43) of flat t: (values f32, indices int64, meta) where
    meta (16 B, device) holds the final threshold for dgc_mask_update.  sample_idx: int64 device
    indices (the reference's CPU uniform_ stream) or None for the device generator."""
    t = dev_f32(t)
    n = t.numel()
    ns = max(1, int(n * 0.01))
    ks = max(1, int(n * ratio * 0.01))
    sample = torch.empty(ns, dtype=F32, device=t.device)
    _lib.call("grace_dgc_sample", _p(t), n, _opt(sample_idx), int(seed) & (2 ** 64 - 1), ns, _p(sample), _stream())
    top, kt = _dgc_sample_top(sample, min(ks, ns))
    ws = workspace("dgc", _lib.query("grace_dgc_workspace_bytes", n), t.device)
    _lib.call("grace_dgc_threshold", _p(t), n, _p(top), kt, float(ratio), _p(ws), _stream())
    meta = ws[:16].clone()
    count = int(meta[8:12].view(torch.int32).item())          # host sync: the payload size
    vals = torch.empty(count, dtype=F32, device=t.device)
    idx = torch.empty(count, dtype=torch.int64, device=t.device)
    if count:
        _lib.call("grace_dgc_write", _p(t), n, _p(ws), _p(vals), _p(idx), _stream())
    return vals, idx, meta


def dgc_threshold_dev(t, ratio, sample_idx=None, seed=0):
    """DgcCompressor.compress's threshold, chunk counts and offsets (grace_dgc_threshold) with NO
    host read: the count stays on the device (meta words: thr0, thr, count at ws[8:12]) for the
    capacity-bounded or counts exchange (grace_amd/dist/compressor/dgc.py)."""
    t = dev_f32(t)
    n = t.numel()
    ns = max(1, int(n * 0.01))
    ks = max(1, int(n * ratio * 0.01))
    sample = torch.empty(ns, dtype=F32, device=t.device)
    _lib.call("grace_dgc_sample", _p(t), n, _opt(sample_idx), int(seed) & (2 ** 64 - 1), ns, _p(sample), _stream())
    top, kt = _dgc_sample_top(sample, min(ks, ns))
    ws = workspace("dgc", _lib.query("grace_dgc_workspace_bytes", n), t.device)
    _lib.call("grace_dgc_threshold", _p(t), n, _p(top), kt, float(ratio), _p(ws), _stream())
    return ws


def dgc_write_capped(t, ws, cap):
    """This rank's exchange record {count, cap | vals f32[cap] | idx i32[cap]} (int32 words)."""
    t = dev_f32(t)
    rec = torch.empty(exchange_record_words(cap), dtype=torch.int32, device=t.device)
    _lib.call("grace_dgc_write_capped", _p(t), t.numel(), _p(ws), _p(rec), int(cap), _stream())
    return rec


def dgc_mask_update_capped(rec, cap, residual, accum):
    _lib.call("grace_dgc_mask_update_capped", _p(rec), int(cap), _p(residual), _p(accum), _stream())


def dgc_select(t, ratio, sample_idx=None, seed=0):
    """The sampled threshold and its adjustment loop only (grace_dgc_select); returns the DGC
    workspace whose first 16 bytes are the meta grace_dgc_step_w1 / dgc_mask_update read."""
    t = dev_f32(t)
    n = t.numel()
    ns = max(1, int(n * 0.01))
    ks = max(1, int(n * ratio * 0.01))
    sample = torch.empty(ns, dtype=F32, device=t.device)
    _lib.call("grace_dgc_sample", _p(t), n, _opt(sample_idx), int(seed) & (2 ** 64 - 1), ns, _p(sample), _stream())
    top, kt = _dgc_sample_top(sample, min(ks, ns))
    ws = workspace("dgc", _lib.query("grace_dgc_workspace_bytes", n), t.device)
    _lib.call("grace_dgc_select", _p(t), n, _p(top), kt, float(ratio), _p(ws), _stream())
    return ws


def dgc_step_w1(t, residual, accum, ws, out=None):
    t = dev_f32(t)
    out = torch.empty_like(t) if out is None else out
    _lib.call("grace_dgc_step_w1", _p(t), _p(residual), _p(accum), t.numel(), _p(ws), _p(out), _stream())
    return out


def dgc_step_w1_fused(g, residual, accum, has_state, momentum, ratio, sample_idx=None, seed=0):
    """World-1 Allgather(DGC, DgcMemory).step from the OLD memory state (grace_dgc_sample_comp +
    grace_dgc_step_w1_fused): returns (out, new residual, new accumulator); the old buffers are only
    read.  Same values as compensate + select + step_w1."""
    g = dev_f32(g)
    n = g.numel()
    ns = max(1, int(n * 0.01))
    ks = max(1, int(n * ratio * 0.01))
    sample = torch.empty(ns, dtype=F32, device=g.device)
    _lib.call("grace_dgc_sample_comp", _p(g), _p(residual) if has_state else None,
              _p(accum) if has_state else None, 1 if has_state else 0, float(momentum), n, _opt(sample_idx),
              int(seed) & (2 ** 64 - 1), ns, _p(sample), _stream())
    top, kt = _dgc_sample_top(sample, min(ks, ns))
    ws = workspace("dgc_w1", _lib.query("grace_dgc_step_w1_fused_workspace_bytes", n), g.device)
    r_new, a_new, out = torch.empty_like(g), torch.empty_like(g), torch.empty_like(g)
    _lib.call("grace_dgc_step_w1_fused", _p(g), _p(residual) if has_state else None,
              _p(accum) if has_state else None, 1 if has_state else 0, float(momentum), n, _p(top), kt,
              float(ratio), _p(ws), _p(r_new), _p(a_new), _p(out), _stream())
    return out, r_new, a_new


def dgc_compensate(g, residual, accum, has_state, momentum):
    _lib.call("grace_dgc_compensate", _p(dev_f32(g)), _p(residual), _p(accum), 1 if has_state else 0,
              float(momentum), g.numel(), _stream())


def dgc_mask_update(t, residual, accum, meta):
    _lib.call("grace_dgc_mask_update", _p(dev_f32(t)), _p(residual), _p(accum), t.numel(), _p(meta), _stream())


def sumsq(x):
    x = dev_f32(x)
    out = torch.empty(1, dtype=F32, device=x.device)
    ws = workspace("sumsq", _lib.query("grace_sumsq_workspace_bytes"), x.device)
    _lib.call("grace_sumsq", _p(x), x.numel(), _p(ws), _p(out), _stream())
    return out


def clip_by_sumsq(x, s, world):
    x = dev_f32(x)
    out = torch.empty_like(x)
    _lib.call("grace_clip_by_sumsq", _p(x), _p(s), float(world), _p(out), x.numel(), _stream())
    return out


# ----------------------------------------------------------------------------- packed wire formats
def pack_bits(codes):
    """u8 {0,1} codes -> int32 words, bit i = code i (LSB first)."""
    codes = require_dev(codes, "codes")
    n = codes.numel()
    words = torch.empty((n + 31) // 32, dtype=torch.int32, device=codes.device)
    _lib.call("grace_pack_bits", _p(codes), n, _p(words), _stream())
    return words


def sign_encode_bits(x):
    """sign codes (x >= 0) of a f32 device tensor straight into int32 words (the pack_bits layout)."""
    x = dev_f32(x)
    n = x.numel()
    words = torch.empty((n + 31) // 32, dtype=torch.int32, device=x.device)
    _lib.call("grace_sign_encode_bits", _p(x), n, _p(words), _stream())
    return words


def unpack_bits(words, n):
    words = require_dev(words, "words")
    codes = torch.empty(n, dtype=torch.uint8, device=words.device)
    _lib.call("grace_unpack_bits", _p(words), n, _p(codes), _stream())
    return codes


def sign_majority_bits(words_wn, world, n):
    words_wn = require_dev(words_wn, "words")
    out = torch.empty(n, dtype=F32, device=words_wn.device)
    _lib.call("grace_sign_majority_bits", _p(words_wn), (n + 31) // 32, int(world), n, _p(out), _stream())
    return out


def pack2(values):
    values = require_dev(values, "values")
    n = values.numel()
    out = torch.empty(_lib.query("grace_pack2_bytes", n), dtype=torch.uint8, device=values.device)
    _lib.call("grace_pack2", _p(values), n, _p(out), _stream())
    return out


def unpack2(packed, n):
    packed = require_dev(packed, "packed")
    out = torch.empty(n, dtype=torch.uint8, device=packed.device)
    _lib.call("grace_unpack2", _p(packed), n, _p(out), _stream())
    return out


def tern_pack(codes):
    codes = require_dev(codes, "codes")
    n = codes.numel()
    out = torch.empty(_lib.query("grace_pack2_bytes", n), dtype=torch.uint8, device=codes.device)
    _lib.call("grace_tern_pack", _p(codes), n, _p(out), _stream())
    return out


def tern_unpack(packed, n):
    packed = require_dev(packed, "packed")
    out = torch.empty(n, dtype=torch.int8, device=packed.device)
    _lib.call("grace_tern_unpack", _p(packed), n, _p(out), _stream())
    return out
