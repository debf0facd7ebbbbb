"""Allgather, Horovod flavour (grace_dl/torch/communicator/allgather.py:7-45), on async
torch.distributed all-gathers.  Variable-size payloads exchange their sizes first (one small
synchronous all-gather, as the reference's ``allgather(tensors_size)``) and are padded to the
largest rank's size for the async gather."""
import torch
import torch.distributed as dist

from grace_amd.dist._util import divide
from grace_amd.torch import Communicator


class Allgather(Communicator):
    def __init__(self, compressor, memory, world_size):
        super().__init__(compressor, memory)
        self.world_size = world_size

    def async_send(self, tensors_compressed, name):
        W = int(self.world_size)
        sizes = [t.numel() for t in tensors_compressed]
        if self.compressor.tensors_size_are_same or W == 1:
            per_rank = [sizes] * W
        else:
            dev = tensors_compressed[0].device
            local = torch.tensor(sizes, dtype=torch.int64, device=dev)
            allsz = torch.empty(W * len(sizes), dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(allsz, local)
            per_rank = allsz.view(W, -1).cpu().tolist()
        handles = []
        for j, t in enumerate(tensors_compressed):
            flat = t.contiguous().view(-1)
            mx = max(per_rank[r][j] for r in range(W))
            if W == 1:
                handles.append((None, flat, mx))
                continue
            if flat.numel() != mx:
                pad = torch.zeros(mx, dtype=flat.dtype, device=flat.device)
                pad[:flat.numel()] = flat
                flat = pad
            out = torch.empty(W * mx, dtype=flat.dtype, device=flat.device)
            work = dist.all_gather_into_tensor(out, flat, async_op=True) if mx else None
            handles.append((work, out, mx))
        return handles, per_rank

    def wait_receive(self, result, ctx):
        handles, per_rank = result
        W = int(self.world_size)
        gathered = []
        for work, out, _ in handles:
            if work is not None:
                work.wait()
            gathered.append(out)
        decompressed = []
        for r in range(W):
            tc = [g.view(W, -1)[r][:per_rank[r][j]] if W > 1 else g for j, g in enumerate(gathered)]
            decompressed.append(self.compressor.decompress(tc, ctx))
        agg = self.compressor.aggregate(decompressed)
        return divide(agg, W) if self.compressor.average else agg
