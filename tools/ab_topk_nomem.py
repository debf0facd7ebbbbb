"""A/B the world-1 top-k step without memory (grace_topk_step_dense, 256 MiB, 1 %) between builds of
libgrace_hip in ONE process: interleaved rounds, per-build median step time and topk_main time (event
timer).  usage: python tools/ab_topk_nomem.py LIB_A LIB_B [...]"""
import ctypes
import statistics
import sys

import torch

libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
P_, I64, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
for L in libs:
    L.grace_topk_step_dense.argtypes = [P_, I64, I64, P_, P_, P_, P_, SZ, P_]
    L.grace_topk_workspace_bytes.restype = SZ
    L.grace_topk_workspace_bytes.argtypes = [I64, I64]
    L.grace_timer_collect.argtypes = [P_, P_]
n = 64 * 1024 * 1024
k = n // 100
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
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
            L.grace_topk_step_dense(gs[s % 3].data_ptr(), n, k, pay.data_ptr(), pay[k:].data_ptr(), out.data_ptr(),
                                    None, ctypes.c_int64(0), wss[i].data_ptr(), wss[i].numel(), stream)
        e1.record()
        torch.cuda.synchronize()
        ms = ctypes.c_float(0)
        cnt = ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd > 0:
            res[i][0].append(e0.elapsed_time(e1) / 10 * 1e3)
            res[i][1].append(ms.value / max(cnt.value, 1) * 1e3)
for i, p in enumerate(sys.argv[1:]):
    print({"lib": p, "step_us_median": round(statistics.median(res[i][0]), 2),
           "main_us_median": round(statistics.median(res[i][1]), 2)})
