"""Can RCCL run 2 ranks on ONE GPU (the gpurun box has one)?  If it can, the W > 1 bench path can be
rehearsed over RCCL instead of gloo.  Run under torch.distributed.run --nproc-per-node 2."""
import os
import sys

import torch
import torch.distributed as dist

dist.init_process_group("nccl")
rank, world = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
x = torch.full((4,), float(rank + 1), device="cuda:0")
out = torch.empty(4 * world, device="cuda:0")
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: {out.tolist()}", flush=True)
dist.destroy_process_group()
sys.exit(0)
