"""Allreduce, Horovod flavour (grace_dl/torch/communicator/allreduce.py:5-17): in-place async
all-reduce of each payload tensor; Horovod's ``allreduce_async_(t, average)`` averages, so the
sum is divided by the world size when the compressor averages."""
import torch.distributed as dist

from grace_amd.dist._util import divide
from grace_amd.torch import Communicator


class Allreduce(Communicator):
    def __init__(self, compressor, memory, world_size=None):
        super().__init__(compressor, memory)
        self.world_size = world_size

    def _world(self):
        if self.world_size is not None:
            return int(self.world_size)
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def async_send(self, tensors_compressed, name):
        W = self._world()
        handles = []
        for t in tensors_compressed:
            work = dist.all_reduce(t, async_op=True) if W > 1 else None
            handles.append((work, t))
        return handles

    def wait_receive(self, handles, ctx):
        W = self._world()
        output = []
        for work, t in handles:
            if work is not None:
                work.wait()
            output.append(divide(t, W) if self.compressor.average and W > 1 else t)
        return self.compressor.decompress(output, ctx)
