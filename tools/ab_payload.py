"""A/B the world > 1 payload grouping (grace_sort_payload) between builds of libgrace_hip in one
process: a 256 MiB top-k 1 % payload (671,088 entries), per-build median over rounds.
usage: python tools/ab_payload.py LIB_A LIB_B [...]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

V, I64 = ctypes.c_void_p, ctypes.c_int64
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_sort_payload.argtypes = [V, V, I64, I64, V, V, V, V, ctypes.c_size_t, V]
n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
pays = []
for j in range(3):
    g = torch.randn(n, device=dev)
    r = torch.zeros(n, device=dev)
    buf, _, _ = ops.topk_residual_step(g, r, True, 1.0, 1.0, k, out=None)
    pays.append(buf.clone())
del g, r
out = torch.empty(2 * k + (n + 8191) // 8192, dtype=torch.float32, device=dev)
ws = [torch.zeros(256, dtype=torch.uint8, device=dev) for _ in libs]
stream = torch.cuda.current_stream().cuda_stream
res = {i: [] for i in range(len(libs))}
for rnd in range(8):
    for i, L in enumerate(libs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for s in range(30):
            p = pays[s % 3]
            L.grace_sort_payload(p.data_ptr(), p[k:].data_ptr(), k, n, out.data_ptr(), out[k:].data_ptr(),
                                 out[2 * k:].data_ptr(), ws[i].data_ptr(), 256, stream)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            res[i].append(e0.elapsed_time(e1) / 30 * 1e3)
for i, p in enumerate(sys.argv[1:]):
    print({"lib": os.path.basename(p), "sort_payload_us": round(statistics.median(res[i]), 2)})
