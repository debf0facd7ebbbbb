"""Step time of the fused top-k 1 % + residual step (256 MiB) with the bench's kernel timer on and
off, interleaved in one process; run under `rocprofv3 --kernel-trace` to see the launch gaps.
usage: python tools/exp_gaps.py"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
k = n // 100
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
rs = [0.1 * torch.randn(n, device=dev) for _ in range(3)]
out = torch.empty(n, device=dev)
res = {False: [], True: []}
for rnd in range(6):
    for timer in (False, True):
        ops.timer_enable(timer)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for s in range(10):
            j = s % 3
            ops.topk_residual_step(gs[j], rs[j], True, 1.0, 1.0, k, out=out)
        e1.record()
        torch.cuda.synchronize()
        if timer:
            ops.timer_collect()
        ops.timer_enable(False)
        if rnd > 0:
            res[timer].append(e0.elapsed_time(e1) / 10 * 1e3)
for t in (False, True):
    print({"timer": t, "step_us_median": round(statistics.median(res[t]), 2), "all": [round(x, 1) for x in res[t]]})
