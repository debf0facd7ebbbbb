"""Is the sporadic fast fused main pass (tools/ab_place3.py: 2 of 12 states at 171-173 us against
188-190 us) a matter of physically contiguous buffers (larger page fragments, fewer translation
misses)?  Buffers from hipExtMallocWithFlags(hipDeviceMallocContiguous) against torch's caching
allocator, for the residual + output only and for all three streams; several states of each kind,
interleaved rounds, median topk_main (the library's dispatch-packet timer).
usage: python tools/ab_contig.py [LIB] [STATES_PER_KIND]"""
import ctypes
import statistics
import sys

import torch

P_, I32, I64, SZ, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
lib = sys.argv[1] if len(sys.argv) > 1 else "grace_amd/lib/libgrace_hip.so"
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
L = ctypes.CDLL(lib)
L.grace_topk_residual_step_carry.argtypes = [P_, P_, I32, F32, F32, I64, I64, P_, P_, P_, P_, I64, I32, P_, I64,
                                             P_, SZ, P_]
L.grace_topk_workspace_bytes.restype = SZ
L.grace_topk_workspace_bytes.argtypes = [I64, I64]
L.grace_timer_collect.argtypes = [P_, P_]
L.grace_last_error.restype = ctypes.c_char_p
H = ctypes.CDLL("libamdhip64.so")
H.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), SZ, ctypes.c_uint]
H.hipExtMallocWithFlags.restype = ctypes.c_int
n = 64 * 1024 * 1024
k = n // 100
dev = torch.device("cuda", 0)
torch.manual_seed(0)


class DevBuf:
    """A raw device allocation seen by torch through __cuda_array_interface__ (kept alive here)."""

    def __init__(self, nelem, flags):
        self.p = ctypes.c_void_p()
        rc = H.hipExtMallocWithFlags(ctypes.byref(self.p), nelem * 4, flags)
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({flags}) failed: {rc}")
        self.__cuda_array_interface__ = {"shape": (nelem,), "typestr": "<f4", "data": (self.p.value, False),
                                         "version": 2, "strides": None}


keep = []


def tens(kind):
    if kind == "torch":
        return torch.empty(n, device=dev)
    b = DevBuf(n, 0x4 if kind == "contig" else 0x0)
    keep.append(b)
    return torch.as_tensor(b, device=dev)


g_torch = [torch.randn(n, device=dev) for _ in range(3)]
g_contig = []
for j in range(3):
    t = tens("contig")
    t.copy_(g_torch[j])
    g_contig.append(t)
stream = torch.cuda.current_stream().cuda_stream
ws = torch.zeros(L.grace_topk_workspace_bytes(n, k), dtype=torch.uint8, device=dev)
vals = torch.zeros(k, device=dev)
idx = torch.zeros(k, dtype=torch.int32, device=dev)
states = []
for s in range(NS):
    for kind, gk in (("torch", "torch"), ("contig", "torch"), ("contig", "contig"), ("hipmalloc", "torch")):
        out = tens(kind)
        out.zero_()
        res = []
        for j in range(3):
            r = tens(kind)
            r.copy_(0.1 * torch.randn(n, device=dev))
            res.append(r)
        states.append((f"r,out {kind:9s} g {gk:6s}", g_contig if gk == "contig" else g_torch, res, out))


def step(st, s):
    _, gs, res, out = st
    j = s % 3
    rc = L.grace_topk_residual_step_carry(gs[j].data_ptr(), res[j].data_ptr(), 1, 1.0, 1.0, n, k, vals.data_ptr(),
                                          idx.data_ptr(), out.data_ptr(), None, 0, 0, None, 0, ws.data_ptr(),
                                          ws.numel(), stream)
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


times = {i: [] for i in range(len(states))}
for rnd in range(5):
    for i, st in enumerate(states):
        L.grace_timer_enable(1)
        torch.cuda.synchronize()
        for s in range(9):
            step(st, s)
        torch.cuda.synchronize()
        ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd >= 1:
            times[i].append(ms.value / max(cnt.value, 1) * 1e3)
    print(f"round {rnd} done", flush=True)
for i, st in enumerate(states):
    b = times[i]
    print(f"{st[0]}  topk_main median {statistics.median(b):6.1f} us (min {min(b):.1f} max {max(b):.1f})  out "
          f"{st[3].data_ptr():#x}", flush=True)
