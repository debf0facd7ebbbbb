"""A/B the world-1 PowerSGD one-pass compress (grace_powersgd_w1_compress: psgd_w1_pass +
psgd_w1_fin) between builds of libgrace_hip in ONE process: interleaved rounds, per-build median
of the compress time (events around 20 back-to-back compresses on 5 rotated 4096 x 4096 matrices)
and a cross-build check that P and Q agree.  usage: python tools/ab_psgd.py LIB_A LIB_B [...]"""
import ctypes
import statistics
import sys

import torch

P_, I64, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_powersgd_w1_compress.argtypes = [P_, I64, I64, P_, ctypes.c_uint64, P_, P_, P_, SZ, P_, P_]
    L.grace_powersgd_w1_workspace_bytes.restype = SZ
    L.grace_powersgd_w1_workspace_bytes.argtypes = [I64, I64]
n = m = 4096
dev = torch.device("cuda", 0)
Ms = [torch.randn(n, m, device=dev) for _ in range(5)]
P = torch.empty(n, 4, device=dev)
Q = torch.empty(m, 4, device=dev)
wss = [torch.zeros(L.grace_powersgd_w1_workspace_bytes(n, m), dtype=torch.uint8, device=dev) for L in libs]
stream = torch.cuda.current_stream().cuda_stream
outs = []
for i, L in enumerate(libs):
    rc = L.grace_powersgd_w1_compress(Ms[0].data_ptr(), n, m, None, 7, P.data_ptr(), Q.data_ptr(),
                                      wss[i].data_ptr(), wss[i].numel(), None, stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    outs.append((P.clone(), Q.clone()))
res = {i: [] for i in range(len(libs))}
for rnd in range(8):
    for i, L in enumerate(libs):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for s in range(20):
            L.grace_powersgd_w1_compress(Ms[s % 5].data_ptr(), n, m, None, s, P.data_ptr(), Q.data_ptr(),
                                         wss[i].data_ptr(), wss[i].numel(), None, stream)
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            res[i].append(e0.elapsed_time(e1) / 20 * 1e3)
for i, p in enumerate(sys.argv[1:]):
    dp = (outs[i][0] - outs[0][0]).abs().max().item()
    dq = (outs[i][1] - outs[0][1]).abs().max().item()
    print({"lib": p, "compress_us_median": round(statistics.median(res[i]), 2), "max_dP_vs_first": dp,
           "max_dQ_vs_first": dq})
