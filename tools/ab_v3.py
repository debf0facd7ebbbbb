"""A/B of top-k main-pass builds of libgrace_hip in ONE process (r06: the v3 classification against
the r05 v2 one), on the 256 MiB bucket at k = 1 %, 3 rotated input sets:
  nomem_rec   Allgather(TopK, NoneMemory).step with the recycled output (grace_topk_step_dense, prev_idx)
  nomem_dense the same with a fresh dense output
  fused       the world-1 top-k + residual step with the dense output (grace_topk_residual_step_carry)
  swap        the W > 1 residual step into a second buffer (grace_topk_residual_step_swap)
Interleaved rounds; per build and mode the median step (events around 10 steps) and the median
topk_main time (the library's dispatch-packet event timer).  Every build's results are compared bit
for bit with the first build's on the same inputs (payload as a sorted set, residual and output).
usage: python tools/ab_v3.py LIB_A LIB_B [...]"""
import ctypes
import statistics
import sys

import torch

P_, I32, I64, SZ, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_topk_step_dense.argtypes = [P_, I64, I64, P_, P_, P_, P_, I64, P_, SZ, P_]
    L.grace_topk_residual_step_carry.argtypes = [P_, P_, I32, F32, F32, I64, I64, P_, P_, P_, P_, I64, I32, P_, I64,
                                                 P_, SZ, P_]
    L.grace_topk_residual_step_swap.argtypes = [P_, P_, I32, F32, F32, I64, I64, P_, P_, P_, P_, I64, I32, P_, SZ, P_]
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
wss = [torch.zeros(L.grace_topk_workspace_bytes(n, k), dtype=torch.uint8, device=dev) for L in libs]


def chk(L, rc):
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


class State:
    """Per build and mode: residuals, outputs and payloads that persist across steps."""

    def __init__(self):
        self.out = torch.zeros(n, device=dev)
        self.vals = [torch.zeros(k, device=dev) for _ in range(3)]
        self.idx = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in range(3)]
        self.res = [0.1 * torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7 + j))
                    for j in range(3)]
        self.res2 = [torch.empty(n, device=dev) for _ in range(3)]
        self.prev = None


def step(i, L, ws, st, mode, s):
    j = s % 3
    if mode == "nomem_rec" or mode == "nomem_dense":
        prev = st.prev if mode == "nomem_rec" and st.prev is not None else None
        chk(L, L.grace_topk_step_dense(gs[j].data_ptr(), n, k, st.vals[j].data_ptr(), st.idx[j].data_ptr(),
                                       st.out.data_ptr(), prev.data_ptr() if prev is not None else None,
                                       k if prev is not None else 0, ws.data_ptr(), ws.numel(), stream))
        st.prev = st.idx[j]
    elif mode == "fused":
        chk(L, L.grace_topk_residual_step_carry(gs[j].data_ptr(), st.res[j].data_ptr(), 1, 1.0, 1.0, n, k,
                                                st.vals[j].data_ptr(), st.idx[j].data_ptr(), st.out.data_ptr(),
                                                None, 0, 0, None, 0, ws.data_ptr(), ws.numel(), stream))
    elif mode == "swap":
        chk(L, L.grace_topk_residual_step_swap(gs[j].data_ptr(), st.res[j].data_ptr(), 1, 1.0, 1.0, n, k,
                                               st.vals[j].data_ptr(), st.idx[j].data_ptr(), st.res2[j].data_ptr(),
                                               None, 0, 0, ws.data_ptr(), ws.numel(), stream))
        st.res[j], st.res2[j] = st.res2[j], st.res[j]


import os
modes = os.environ.get("AB_MODES", "nomem_rec,nomem_dense,fused,swap").split(",")
# bit-exactness across builds: 4 steps of every mode from the same start
ref = {}
for i, L in enumerate(libs):
    for mode in modes:
        st = State()
        for s in range(4):
            step(i, L, wss[i], st, mode, s)
        torch.cuda.synchronize()
        j = 3 % 3
        got = (torch.sort(st.idx[j].long())[0].cpu(), st.out.cpu(), st.res[j].cpu())
        key = mode
        if i == 0:
            ref[key] = got
        else:
            same = all(torch.equal(a, b) if a.dtype != torch.float32 else torch.equal(a.view(torch.int32), b.view(torch.int32))
                       for a, b in zip(ref[key], got))
            print(f"bit-exact {sys.argv[1 + i].rsplit('/', 1)[-1]} vs {sys.argv[1].rsplit('/', 1)[-1]} {mode}: {same}",
                  flush=True)
res = {(i, m): ([], []) for i in range(len(libs)) for m in modes}
states = {(i, m): State() for i in range(len(libs)) for m in modes}
for rnd in range(6):
    for mode in modes:
        for i, L in enumerate(libs):
            st = states[(i, mode)]
            L.grace_timer_enable(1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(10):
                step(i, L, wss[i], st, mode, s)
            e1.record()
            torch.cuda.synchronize()
            ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
            L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
            L.grace_timer_enable(0)
            if rnd >= 1:
                res[(i, mode)][0].append(e0.elapsed_time(e1) / 10 * 1e3)
                res[(i, mode)][1].append(ms.value / max(cnt.value, 1) * 1e3)
for mode in modes:
    for i in range(len(libs)):
        a, b = res[(i, mode)]
        print(f"{mode:12s} {sys.argv[1 + i].rsplit('/', 1)[-1]:28s} step {statistics.median(a):7.1f} us  "
              f"topk_main {statistics.median(b):7.1f} us", flush=True)
