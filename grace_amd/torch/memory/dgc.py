"""DgcMemory, Horovod flavour (grace_dl/torch/memory/dgc.py:7-38): same momentum correction as the dist
copy; the constructor has no world_size and clipping uses ``sqrt(allreduce_(sum(g*g), average=True))``
(which works here, where the dist copy's ``dist.all_reduce`` returns None and raises)."""
import torch.distributed as dist

from grace_amd.dist.memory.dgc import DgcMemory as _DistDgcMemory


class DgcMemory(_DistDgcMemory):
    def __init__(self, momentum, gradient_clipping):
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        super().__init__(momentum, gradient_clipping, world)
