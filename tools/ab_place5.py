"""Placement probe, fifth form: which buffer carries a fast placement -- the residuals or the dense
output?  States as tools/ab_place3.py builds them; every state timed with its own buffers, with its
residuals and state 0's output, and with state 0's residuals and its output (median topk_main over
interleaved rounds).
usage: python tools/ab_place5.py [LIB] [STATES]"""
import ctypes
import statistics
import sys

import torch

P_, I32, I64, SZ, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
lib = sys.argv[1] if len(sys.argv) > 1 else "grace_amd/lib/libgrace_hip.so"
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 12
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


class State:
    def __init__(self):
        self.out = torch.zeros(n, device=dev)
        self.vals = [torch.zeros(k, device=dev) for _ in range(3)]
        self.idx = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in range(3)]
        self.res = [0.1 * torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7 + j))
                    for j in range(3)]
        self.res2 = [torch.empty(n, device=dev) for _ in range(3)]


def step(st, s):
    j = s % 3
    rc = L.grace_topk_residual_step_carry(gs[j].data_ptr(), st.res[j].data_ptr(), 1, 1.0, 1.0, n, k,
                                          st.vals[j].data_ptr(), st.idx[j].data_ptr(), st.out.data_ptr(), None, 0, 0,
                                          None, 0, ws.data_ptr(), ws.numel(), stream)
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


for c in range(4):   # churn: states allocated, stepped and freed (ab_v3's bit-exactness phase)
    st = State()
    for s in range(4):
        step(st, s)
    torch.cuda.synchronize()
    del st
states = [State() for _ in range(NS)]


class Mix:
    """residuals of one state with the output of another"""

    def __init__(self, a, b):
        self.res, self.vals, self.idx, self.out = a.res, a.vals, a.idx, b.out


combos = [("own", i, i) for i in range(NS)] + [("res_i+out_0", i, 0) for i in range(1, NS)] + \
         [("res_0+out_i", 0, i) for i in range(1, NS)]
times = {c: [] for c in range(len(combos))}
for rnd in range(5):
    for c, (tag, i, j) in enumerate(combos):
        st = Mix(states[i], states[j])
        L.grace_timer_enable(1)
        torch.cuda.synchronize()
        for s in range(6):
            step(st, s)
        torch.cuda.synchronize()
        ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd >= 1:
            times[c].append(ms.value / max(cnt.value, 1) * 1e3)
    print(f"round {rnd} done", flush=True)
for c, (tag, i, j) in enumerate(combos):
    print(f"{tag:12s} res of {i:2d}, out of {j:2d}: topk_main median {statistics.median(times[c]):6.1f} us", flush=True)
