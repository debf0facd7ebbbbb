"""Broadcast communicator (grace_dl/dist/communicator/broadcast.py:7-33): every rank broadcasts its
payload in turn; decode each, aggregate, average.  ``rank`` defaults to the process-group rank
(the reference's helper omits it and raises TypeError, grace_dl/dist/helper.py:95-97)."""
import torch
import torch.distributed as dist

from grace_amd.dist import Communicator
from grace_amd.dist._util import divide


class Broadcast(Communicator):

    def __init__(self, compressor, memory, world_size, rank=None):
        super().__init__(compressor, memory, world_size)
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.rank = rank

    def send_receive(self, tensors, name, ctx):
        if not self.compressor.tensors_size_are_same:
            raise NotImplementedError("Broadcast needs same-size payloads (broadcast.py:14-15)")
        W = int(self.world_size)
        tensors_decompressed = []
        for root_rank in range(W):
            if root_rank == self.rank:
                broadcasted = list(tensors)
                if W > 1:
                    for t in broadcasted:
                        dist.broadcast(t, root_rank)
            else:
                broadcasted = []
                for t in tensors:
                    recv = torch.empty_like(t)
                    dist.broadcast(recv, root_rank)
                    broadcasted.append(recv)
            tensors_decompressed.append(self.compressor.decompress(broadcasted, ctx))
        tensor_aggregated = self.compressor.aggregate(tensors_decompressed)
        return divide(tensor_aggregated, W) if self.compressor.average else tensor_aggregated
