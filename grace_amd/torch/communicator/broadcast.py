"""Broadcast, Horovod flavour (grace_dl/torch/communicator/broadcast.py:5-30): every rank
broadcasts its payload (async), each is decompressed with the local ctx and aggregated."""
import torch
import torch.distributed as dist

from grace_amd.dist._util import divide
from grace_amd.torch import Communicator


class Broadcast(Communicator):
    def __init__(self, compressor, memory, world_size):
        super().__init__(compressor, memory)
        self.world_size = world_size

    def async_send(self, tensors_compressed, name):
        W = int(self.world_size)
        rank = dist.get_rank() if W > 1 else 0
        handles = []
        for root in range(W):
            rank_handles = []
            for t in tensors_compressed:
                buf = t.clone() if root == rank else torch.empty_like(t)
                work = dist.broadcast(buf, root, async_op=True) if W > 1 else None
                rank_handles.append((work, buf))
            handles.append(rank_handles)
        return handles

    def wait_receive(self, handles, ctx):
        W = int(self.world_size)
        decompressed = []
        for rank_handles in handles:
            tensors = []
            for work, buf in rank_handles:
                if work is not None:
                    work.wait()
                tensors.append(buf)
            decompressed.append(self.compressor.decompress(tensors, ctx))
        agg = self.compressor.aggregate(decompressed)
        return divide(agg, W) if self.compressor.average else agg
