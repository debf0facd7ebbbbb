"""Time the top-k step on degenerate buckets that force the exact fallback (massive ties):
256 MiB, 99.75 % zeros and all-equal, with residual memory.  Run on the GPU box."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
g = torch.zeros(n, device=dev)
idx = torch.randperm(n, device=dev)[: n // 400]
g[idx] = torch.randn(idx.numel(), device=dev)
cases = {"sparse_99.75pct_zeros": g, "constant": torch.full((n,), 0.5, device=dev),
         "normal": torch.randn(n, device=dev)}
for name, x in cases.items():
    r = torch.zeros(n, device=dev)
    out = torch.empty(n, device=dev)
    for _ in range(2):
        ops.topk_residual_step(x, r, True, 1.0, 1.0, k, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.topk_residual_step(x, r, True, 1.0, 1.0, k, out=out)
    e1.record()
    torch.cuda.synchronize()
    print({"case": name, "ms_per_step": round(e0.elapsed_time(e1) / 5, 3), "status": ops.topk_status(n, k, dev)})
