"""Does where a step's buffers land in HBM change the headline step time?  
The same Allgather(TopK 1 %, ResidualMemory).step sequence over the same three 256 MiB gradients,
with SETS independent communicators (each has its own residual and output buffers, allocated one
after the other), on one stream, interleaved rounds in one process: per-set median ms per step.
A spread between sets that holds across rounds is a property of the buffers, not of the code.
usage: python tools/exp_placement.py [--sets 6] [--rounds 6] [--steps 30]"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.dist.communicator.allgather import Allgather  # noqa: E402
from grace_amd.dist.compressor.topk import TopKCompressor  # noqa: E402
from grace_amd.dist.memory.residual import ResidualMemory  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--numel", type=int, default=1 << 26)
ap.add_argument("--sets", type=int, default=6)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--steps", type=int, default=30)
args = ap.parse_args()

dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev)
grads = []
for j in range(3):
    gen.manual_seed(j + 1)
    grads.append(torch.randn(args.numel, device=dev, generator=gen))
comms = [Allgather(TopKCompressor(0.01), ResidualMemory(), 1) for _ in range(args.sets)]
keep = []


def run(c, steps):
    for i in range(steps):
        keep.append(c.step(grads[i % 3], f"b{i % 3}"))
        if len(keep) > 3:
            keep.pop(0)


for c in comms:                      # allocate every set's residuals and outputs up front
    run(c, 6)
torch.cuda.synchronize()
res = [[] for _ in comms]
for rnd in range(args.rounds):
    for s, c in enumerate(comms):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(c, args.steps)
        torch.cuda.synchronize()
        res[s].append((time.perf_counter() - t0) / args.steps * 1e3)
med = [statistics.median(r) for r in res]
for s, r in enumerate(res):
    print({"set": s, "ms_per_step": round(med[s], 4), "rounds": [round(x, 4) for x in r]}, flush=True)
print({"spread_max_over_min": round(max(med) / min(med), 4)}, flush=True)
