"""A/B the fused top-k + residual step between two builds of libgrace_hip in ONE process on one
device (cdna_hip_programming.md rule 24): interleaved rounds, per-build median of the step time
and of the dominant kernel (event timer).  usage: python tools/ab_topk.py LIB_A LIB_B [...]"""
import ctypes
import statistics
import sys

import torch

libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_topk_residual_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]
    L.grace_topk_workspace_bytes.restype = ctypes.c_size_t
    L.grace_topk_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.grace_timer_collect.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
n = 64 * 1024 * 1024
k = n // 100
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
rs = [0.1 * torch.randn(n, device=dev) for _ in range(3)]
out = torch.empty(n, device=dev)
pay = torch.empty(2 * k, device=dev)
wss = [torch.zeros(L.grace_topk_workspace_bytes(n, k), dtype=torch.uint8, device=dev) for L in libs]
stream = torch.cuda.current_stream().cuda_stream
res = {i: ([], []) for i in range(len(libs))}
for rnd in range(6):
    for i, L in enumerate(libs):
        L.grace_timer_enable(1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for s in range(10):
            j = s % 3
            L.grace_topk_residual_step(gs[j].data_ptr(), rs[j].data_ptr(), 1, 1.0, 1.0, n, k, pay.data_ptr(),
                                       pay[k:].data_ptr(), out.data_ptr(), wss[i].data_ptr(), wss[i].numel(), stream)
        e1.record()
        torch.cuda.synchronize()
        ms = ctypes.c_float(0); cnt = ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd > 0:
            res[i][0].append(e0.elapsed_time(e1) / 10 * 1e3)
            res[i][1].append(ms.value / max(cnt.value, 1) * 1e3)
for i, p in enumerate(sys.argv[1:]):
    print({"lib": p, "step_us_median": round(statistics.median(res[i][0]), 2),
           "main_us_median": round(statistics.median(res[i][1]), 2)})
