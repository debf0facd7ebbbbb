"""grace_from_params for the Horovod flavour (grace_dl/torch/helper.py:1-90): same keys and
defaults; the world size comes from torch.distributed instead of ``hvd.size()``."""
import torch.distributed as dist


def grace_from_params(params):
    from grace_amd.dist.helper import grace_from_params as dist_grace
    world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    p = dict(params)
    p.setdefault('world_size', world_size)
    comm = p.get('communicator', 'allreduce')
    p['communicator'] = 'allreduce'          # build compressor + memory through the shared factory
    built = dist_grace(p)
    compressor, memory = built.compressor, built.memory
    if comm == 'allreduce':
        from grace_amd.torch.communicator.allreduce import Allreduce
        return Allreduce(compressor, memory, p['world_size'])
    if comm == 'allgather':
        from grace_amd.torch.communicator.allgather import Allgather
        return Allgather(compressor, memory, p['world_size'])
    if comm == 'broadcast':
        from grace_amd.torch.communicator.broadcast import Broadcast
        return Broadcast(compressor, memory, p['world_size'])
    raise NotImplementedError(comm)


class DistributedOptimizer:
    """Horovod-style wrapper: each parameter's gradient is sent (send_step) from its autograd hook
    as soon as it is ready and received (receive_step) in ``step()``, so the compressed exchange
    overlaps the rest of the backward pass."""

    def __init__(self, optimizer, grace, named_parameters):
        self.optimizer = optimizer
        self.grace = grace
        self._pending = {}
        self._hooks = []
        for name, p in named_parameters:
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(name)))

    def _make_hook(self, name):
        def hook(p):
            self._pending[name] = (p, self.grace.send_step(p.grad, name))
        return hook

    def synchronize(self):
        for name, (p, (handles, ctx)) in list(self._pending.items()):
            p.grad = self.grace.receive_step(handles, ctx).view(p.grad.shape)
        self._pending.clear()

    def step(self, closure=None):
        self.synchronize()
        return self.optimizer.step(closure)

    def zero_grad(self, set_to_none=True):
        return self.optimizer.zero_grad(set_to_none=set_to_none)
