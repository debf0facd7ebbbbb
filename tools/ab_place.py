"""Does buffer placement move the fused top-k main pass?  ONE build of libgrace_hip, several
independent states (residual r and dense output out, each its own 256 MiB allocation, with a
varying spacer allocated before each) on the same three gradient sets; interleaved rounds, per state
the median step and topk_main time (the library's dispatch-packet timer) and the buffers' device
addresses, so that a slow state can be matched to how its r / out sit relative to g.
usage: python tools/ab_place.py [LIB] [STATES]"""
import ctypes
import os
import statistics
import sys

import torch

P_, I32, I64, SZ, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
lib = sys.argv[1] if len(sys.argv) > 1 else "grace_amd/lib/libgrace_hip.so"
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 6
L = ctypes.CDLL(lib)
L.grace_topk_residual_step_carry.argtypes = [P_, P_, I32, F32, F32, I64, I64, P_, P_, P_, P_, I64, I32, P_, I64,
                                             P_, SZ, P_]
L.grace_topk_workspace_bytes.restype = SZ
L.grace_topk_workspace_bytes.argtypes = [I64, I64]
L.grace_timer_collect.argtypes = [P_, P_]
L.grace_last_error.restype = ctypes.c_char_p
n = 64 * 1024 * 1024
k = n // 100
dev = torch.device("cuda", 0)
torch.manual_seed(0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
stream = torch.cuda.current_stream().cuda_stream
ws = torch.zeros(L.grace_topk_workspace_bytes(n, k), dtype=torch.uint8, device=dev)
spacers = []
states = []
for s in range(NS):
    # spacer: 0, 1, 2, ... MiB + 64 KiB steps, so that r and out land at different offsets
    spacers.append(torch.empty((s * (1 << 20) + s * 65536) // 4 + 1, device=dev))
    r = 0.1 * torch.randn(n, device=dev)
    spacers.append(torch.empty((s * 3 * 65536) // 4 + 1, device=dev))
    out = torch.zeros(n, device=dev)
    vals = torch.zeros(k, device=dev)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    states.append((r, out, vals, idx))


def step(st, j):
    r, out, vals, idx = st
    rc = L.grace_topk_residual_step_carry(gs[j].data_ptr(), r.data_ptr(), 1, 1.0, 1.0, n, k, vals.data_ptr(),
                                          idx.data_ptr(), out.data_ptr(), None, 0, 0, None, 0, ws.data_ptr(),
                                          ws.numel(), stream)
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


res = {s: ([], []) for s in range(NS)}
for rnd in range(7):
    for s in range(NS):
        L.grace_timer_enable(1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(10):
            step(states[s], i % 3)
        e1.record()
        torch.cuda.synchronize()
        ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd >= 1:
            res[s][0].append(e0.elapsed_time(e1) / 10 * 1e3)
            res[s][1].append(ms.value / max(cnt.value, 1) * 1e3)
print("g addresses: " + " ".join(hex(g.data_ptr()) for g in gs), flush=True)
for s in range(NS):
    r, out = states[s][0], states[s][1]
    a, b = res[s]
    print(f"state {s}: r {r.data_ptr():#x} out {out.data_ptr():#x}  (r - g0) mod 16 MiB {(r.data_ptr() - gs[0].data_ptr()) % (1 << 24):#x}"
          f"  (out - r) mod 16 MiB {(out.data_ptr() - r.data_ptr()) % (1 << 24):#x}   step {statistics.median(a):7.1f} us"
          f"  topk_main {statistics.median(b):7.1f} us  (min {min(b):.1f}, max {max(b):.1f})", flush=True)
