"""Placement probe, fourth form: which buffer's placement makes a fused main pass fast, and does a
sub-allocation offset change it?  States as tools/ab_place3.py builds them, but the residuals and the
output are views at offset d into allocations of n + 1 Mi elements: for every state, the pass timed
with (r, out) offsets (0, 0), (64 KiB, 0), (1 MiB, 0), (3 MiB, 0), (0, 64 KiB), (0, 1 MiB), (0, 3 MiB).
If a state's speed follows its offsets, the streams' relative physical placement decides (an engine
could pick its residual's offset); if it does not, the buffers' own pages do.
usage: python tools/ab_place4.py [LIB] [STATES]"""
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
PAD = 1 << 20
k = n // 100
dev = torch.device("cuda", 0)
torch.manual_seed(0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
stream = torch.cuda.current_stream().cuda_stream
ws = torch.zeros(L.grace_topk_workspace_bytes(n, k), dtype=torch.uint8, device=dev)
vals = torch.zeros(k, device=dev)
idx = torch.zeros(k, dtype=torch.int32, device=dev)
OFFS = [(0, 0), (16384, 0), (262144, 0), (786432, 0), (0, 16384), (0, 262144), (0, 786432)]   # elements


class State:
    def __init__(self):
        self.out = torch.zeros(n + PAD, device=dev)
        self.res = []
        for j in range(3):
            t = torch.empty(n + PAD, device=dev)
            t.copy_(0.1 * torch.randn(n + PAD, device=dev))
            self.res.append(t)


def step(st, s, ro, oo):
    j = s % 3
    r = st.res[j]
    rc = L.grace_topk_residual_step_carry(gs[j].data_ptr(), r.data_ptr() + 4 * ro, 1, 1.0, 1.0, n, k,
                                          vals.data_ptr(), idx.data_ptr(), st.out.data_ptr() + 4 * oo, None, 0, 0,
                                          None, 0, ws.data_ptr(), ws.numel(), stream)
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


for c in range(4):
    st = State()
    for s in range(3):
        step(st, s, 0, 0)
    torch.cuda.synchronize()
    del st
states = [State() for _ in range(NS)]
times = {(i, q): [] for i in range(NS) for q in range(len(OFFS))}
for rnd in range(4):
    for i, st in enumerate(states):
        for q, (ro, oo) in enumerate(OFFS):
            L.grace_timer_enable(1)
            torch.cuda.synchronize()
            for s in range(6):
                step(st, s, ro, oo)
            torch.cuda.synchronize()
            ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
            L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
            L.grace_timer_enable(0)
            if rnd >= 1:
                times[(i, q)].append(ms.value / max(cnt.value, 1) * 1e3)
    print(f"round {rnd} done", flush=True)
print("offsets (r, out) in bytes: " + "  ".join(f"({4 * r}, {4 * o})" for r, o in OFFS), flush=True)
for i in range(NS):
    print(f"state {i:2d}: " + "  ".join(f"{statistics.median(times[(i, q)]):6.1f}" for q in range(len(OFFS))), flush=True)
