"""ShardedTopK step times at W = 2 over gloo on one GPU (the N = 2 rehearsal's nested leg), per mode:
replicated / shard dense output, recycled output on / off; host wall time per step after a
device synchronize.  Run under torch.distributed.run with GRACE_BENCH_ONE_DEVICE semantics (both
ranks on cuda:0)."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.dist.sharded import ShardedTopK  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n = 1 << 26
m = n // world
g = torch.randn(m, device=dev)
gs = [torch.randn(m, device=dev) for _ in range(3)]
for dense in ("replicated", "shard"):   # as bench_topk_sharded: 3 names rotated, both engines alive
    for recycle in (True, False):
        eng = ShardedTopK(0.001, dense=dense, recycle_output=recycle)
        ts = []
        for i in range(12):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            eng.step(gs[i % 3], f"{dense[0]}{i % 3}")
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        if rank == 0:
            print(f"dense={dense} recycle={recycle}: ms per step {[round(t, 2) for t in ts]}", flush=True)
dist.destroy_process_group()
