"""A/B in one process: the fused top-k + residual step (256 MiB, 1 %) with and without the
residual-sample carry (grace_topk_residual_step_carry), interleaved rounds over 3 rotated buckets,
median step time and topk_main time (event timer).  usage: python tools/ab_carry.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
variants = {"plain": None, "carry": True}
state = {}
for name in variants:
    rs = [torch.empty(n, device=dev) for _ in range(3)]
    cs = [torch.empty(ops.topk_carry_size(n, k), device=dev) for _ in range(3)]
    state[name] = (rs, cs, [False] * 3)
out = torch.empty(n, device=dev)


def run(name, steps, first=False):
    rs, cs, valid = state[name]
    for s in range(steps):
        j = s % 3
        if variants[name]:
            ops.topk_residual_step(gs[j], rs[j], not first, 1.0, 1.0, k, out=out, carry=cs[j], carry_valid=valid[j])
            valid[j] = True
        else:
            ops.topk_residual_step(gs[j], rs[j], not first, 1.0, 1.0, k, out=out)


for name in variants:
    run(name, 3, first=True)
    run(name, 6)
res = {name: ([], []) for name in variants}
for rnd in range(8):
    for name in variants:
        ops.timer_enable(True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(name, 12)
        e1.record()
        torch.cuda.synchronize()
        main_ms, launches = ops.timer_collect()
        ops.timer_enable(False)
        if rnd > 0:
            res[name][0].append(e0.elapsed_time(e1) / 12 * 1e3)
            res[name][1].append(main_ms / max(launches, 1) * 1e3)
for name in variants:
    print({"variant": name, "step_us_median": round(statistics.median(res[name][0]), 2),
           "step_us_min": round(min(res[name][0]), 2),
           "main_us_median": round(statistics.median(res[name][1]), 2)})
print({"fallback_taken_last": ops.topk_status(n, k, dev)})
