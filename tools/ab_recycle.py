"""A/B in one process: the world-1 top-k step (BASELINE configs[1] and the no-memory step) with the
recycled output vs a fresh dense output every step.  Interleaved rounds of 10 steps over 3 rotated
256 MiB buckets per mode, ms per step (median over rounds), and the main pass's event time."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402
from grace_amd.dist.communicator.allgather import Allgather  # noqa: E402
from grace_amd.dist.compressor.topk import TopKCompressor  # noqa: E402
from grace_amd.dist.memory.none import NoneMemory  # noqa: E402
from grace_amd.dist.memory.residual import ResidualMemory  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 26
gen = torch.Generator(device=dev)
grads = []
for j in range(3):
    gen.manual_seed(j + 1)
    grads.append(torch.randn(n, device=dev, generator=gen))
for mem_cls in (ResidualMemory, NoneMemory):
    comms = {m: Allgather(TopKCompressor(0.01, recycle_output=("always" if m == "recycled" else False)), mem_cls(), 1)
             for m in ("recycled", "dense")}
    res = {m: ([], []) for m in comms}
    for i in range(6):
        for m, c in comms.items():
            c.step(grads[i % 3], f"b{i % 3}")
    for rnd in range(8):
        for m, c in comms.items():
            torch.cuda.synchronize()
            ops.timer_enable(True)
            t0 = time.perf_counter()
            for i in range(10):
                c.step(grads[i % 3], f"b{i % 3}")
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            ms, cnt = ops.timer_collect()
            ops.timer_enable(False)
            res[m][0].append(dt * 1e3)
            res[m][1].append(ms / max(cnt, 1) * 1e3)
    print(mem_cls.__name__, {m: {"ms_per_step": round(statistics.median(v[0]), 4),
                                 "main_us": round(statistics.median(v[1]), 1)} for m, v in res.items()},
          "recycled hits", comms["recycled"].compressor._recycler.hits)

from grace_amd.dist.compressor.randomk import RandomKCompressor  # noqa: E402
comms = {m: Allgather(RandomKCompressor(0.01, recycle_output=(m == "recycled")), ResidualMemory(), 1)
         for m in ("recycled", "dense")}
res = {m: [] for m in comms}
for i in range(6):
    for m, c in comms.items():
        c.step(grads[i % 3], f"b{i % 3}")
for rnd in range(8):
    for m, c in comms.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(10):
            c.step(grads[i % 3], f"b{i % 3}")
        torch.cuda.synchronize()
        res[m].append((time.perf_counter() - t0) / 10 * 1e3)
print("RandomK", {m: round(statistics.median(v), 4) for m, v in res.items()})
