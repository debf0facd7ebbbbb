"""The main pass by dense mode on the 256 MiB headline bucket (k = 1 %), one process, 3 rotated
buffer sets (more than the Infinity Cache holds): the world-1 fused step (g, r read; r', out
written: 16 B per element), the world > 1 step into a second residual buffer (g, r read; r'
written: 12 B), the in-place residual step (12 B), and the stream probe (topk_main with the
classification compiled out) in its 16 B and 12 B layouts.  Run under rocprofv3 --kernel-trace
--stats for per-kernel durations; prints event-timed whole calls.  Usage: python tools/exp_main_modes.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import _lib, ops  # noqa: E402

n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
rs = [0.1 * torch.randn(n, device=dev) for _ in range(3)]
r2 = [torch.empty_like(r) for r in rs]
outs = [torch.empty(n, device=dev) for _ in range(3)]
pws = torch.zeros(int(_lib.query("grace_topk_stream_probe_workspace_bytes", n)), dtype=torch.uint8, device=dev)


def probe(j, sparse):
    _lib.call("grace_topk_stream_probe", gs[j].data_ptr(), rs[j].data_ptr(), outs[j].data_ptr(), n, sparse,
              pws.data_ptr(), pws.numel(), ops._stream())


def fused(j):
    ops.topk_residual_step(gs[j], rs[j], True, 1.0, 1.0, k, out=outs[j])


def swap(j):
    ops.topk_residual_step_swap(gs[j], rs[j], True, 1.0, 1.0, k, r2[j])
    rs[j], r2[j] = r2[j], rs[j]


def inplace(j):
    ops.topk_residual_step(gs[j], rs[j], True, 1.0, 1.0, k, out=None)


cases = {"fused16": fused, "swap12": swap, "inplace12": inplace,
         "probe16": lambda j: probe(j, 0), "probe12": lambda j: probe(j, 1)}
res = {c: [] for c in cases}
for rnd in range(8):
    for c, fn in cases.items():
        for j in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn(j)
            b.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                res[c].append(a.elapsed_time(b) * 1e3)
print({c: round(statistics.median(v), 1) for c, v in res.items()}, flush=True)
