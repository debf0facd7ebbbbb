"""Diagnostic: host-side cost of Allreduce(PowerSGD rank 4, NoneMemory).step on 4096 x 4096 (bench.py
--workload powersgd) against its wall time, plus the kernels alone (no Python between launches)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402
from grace_amd.dist.communicator.allreduce import Allreduce  # noqa: E402
from grace_amd.dist.compressor.powersgd import PowerSGDCompressor  # noqa: E402
from grace_amd.dist.memory.none import NoneMemory  # noqa: E402

dev = torch.device("cuda", 0)
n = m = 4096
Ms = [torch.randn(n, m, device=dev) for _ in range(5)]
comm = Allreduce(PowerSGDCompressor(rank=4, world_size=1), NoneMemory(), 1)
comm_unfused = Allreduce(PowerSGDCompressor(rank=4, world_size=1, one_pass=False), NoneMemory(), 1)
N = 200


def host_us(fn):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(N):
        fn(i)
    h = (time.perf_counter() - t) / N * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / N * 1e6
    return {"host_us": round(h, 2), "wall_us": round(wall, 2)}


P = torch.empty(n, 4, device=dev)
out = torch.empty(n, m, device=dev)


def kernels(i):
    p, q = ops.powersgd_w1_compress(Ms[i % 5], seed=i)
    ops.powersgd_outer(p, q)


print({"comm.step": host_us(lambda i: comm.step(Ms[i % 5], "w")),
       "comm.step unfused": host_us(lambda i: comm_unfused.step(Ms[i % 5], "w")),
       "comm.step again": host_us(lambda i: comm.step(Ms[i % 5], "w")), "w1+outer": host_us(kernels),
       "w1 only": host_us(lambda i: ops.powersgd_w1_compress(Ms[i % 5], seed=i))})
