"""Does the fast/slow placement seen for the fused top-k step (4 streams) exist for a two-stream codec
step (g read, out written: the world-1 signSGD step, ops.launch_sign_step_w1)?  For spacers of S GiB
between g and three output candidates, the median of 10 timed steps per candidate, two rounds.
usage: python tools/ab_out_place.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
dev = torch.device("cuda", 0)
g = torch.randn(n, device=dev)


def timed(out):
    ts = []
    for rep in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.launch_sign_step_w1(g, out)
        e1.record()
        e1.synchronize()
        if rep >= 2:
            ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


for rnd in range(2):
    for S in [0, 1, 2, 3, 4, 5, 6, 8]:
        sp = torch.empty(S << 28, device=dev) if S else None
        outs = [torch.empty(n, device=dev) for _ in range(3)]
        us = [timed(o) for o in outs]
        print(f"round {rnd} spacer {S} GiB: sign step us per output candidate " + " ".join(f"{u:6.1f}" for u in us),
              flush=True)
        del sp, outs
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
