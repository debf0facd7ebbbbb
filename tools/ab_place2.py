"""Placement probe, second form: does the fused top-k main pass (16 B per element: g, r read; r', out
written) run faster for some relative placements of its buffers?  ONE build, one process, the same
three gradients.  States of two kinds, all timed in interleaved rounds (median topk_main by the
library's dispatch-packet timer):
  sep  r and out as separate 256 MiB allocations, with a random-size spacer allocated between them;
  one  r and out carved from ONE allocation of 2n + d elements: out = [0, n), r = [n + d, 2n + d),
       for a set of offsets d (bytes 4 d) -- within one allocation the relative placement is fixed.
usage: python tools/ab_place2.py [LIB] [SEP_STATES]"""
import ctypes
import statistics
import sys

import torch

P_, I32, I64, SZ, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
lib = sys.argv[1] if len(sys.argv) > 1 else "grace_amd/lib/libgrace_hip.so"
NSEP = int(sys.argv[2]) if len(sys.argv) > 2 else 8
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
gen = torch.Generator().manual_seed(11)
keep = []
states = []
for s in range(NSEP):
    r = 0.1 * torch.randn(n, device=dev)
    keep.append(torch.empty(int(torch.randint(1, 64, (1,), generator=gen)) << 18, device=dev))   # 1..63 MiB
    out = torch.zeros(n, device=dev)
    states.append(("sep", s, r, out))
for d in [0, 1024, 16384, 262144, 524288, 1 << 20, 3 << 19]:   # elements: 0, 4 KiB, 64 KiB, 1, 2, 4, 6 MiB
    big = torch.zeros(2 * n + d, device=dev)
    out = big[:n]
    r = big[n + d:2 * n + d]
    r.copy_(0.1 * torch.randn(n, device=dev))
    states.append(("one", d * 4, r, out))
vals = torch.zeros(k, device=dev)
idx = torch.zeros(k, dtype=torch.int32, device=dev)


def step(st, j):
    _, _, r, out = st
    rc = L.grace_topk_residual_step_carry(gs[j].data_ptr(), r.data_ptr(), 1, 1.0, 1.0, n, k, vals.data_ptr(),
                                          idx.data_ptr(), out.data_ptr(), None, 0, 0, None, 0, ws.data_ptr(),
                                          ws.numel(), stream)
    if rc != 0:
        raise RuntimeError(L.grace_last_error().decode())


res = {i: [] for i in range(len(states))}
for rnd in range(5):
    for i, st in enumerate(states):
        L.grace_timer_enable(1)
        torch.cuda.synchronize()
        for s in range(9):
            step(st, s % 3)
        torch.cuda.synchronize()
        ms, cnt = ctypes.c_float(0), ctypes.c_int32(0)
        L.grace_timer_collect(ctypes.addressof(ms), ctypes.addressof(cnt))
        L.grace_timer_enable(0)
        if rnd >= 1:
            res[i].append(ms.value / max(cnt.value, 1) * 1e3)
    print(f"round {rnd} done", flush=True)
g0 = gs[0].data_ptr()
print("g: " + " ".join(hex(g.data_ptr()) for g in gs), flush=True)
for i, (kind, tag, r, out) in enumerate(states):
    b = res[i]
    print(f"{kind} {tag:>8}: r {r.data_ptr():#x} out {out.data_ptr():#x} (r-out) {r.data_ptr() - out.data_ptr():#x}"
          f"  topk_main median {statistics.median(b):6.1f} us (min {min(b):.1f} max {max(b):.1f})", flush=True)
