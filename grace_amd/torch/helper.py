"""grace_from_params for the Horovod flavour (grace_dl/torch/helper.py:1-90): same keys and
defaults, Horovod-flavour codecs; the world size comes from torch.distributed instead of
``hvd.size()``."""
import torch.distributed as dist


def grace_from_params(params):
    """grace_dl/torch/helper.py:1-90 with the Horovod-flavour classes of grace_amd.torch (same keys and
    defaults; powersgd takes no arguments and its rank comes from the memory's compress_rank)."""
    world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    comp = params.get('compressor', 'none')
    mem = params.get('memory', 'none')
    comm = params.get('communicator', 'allreduce')
    if comp == 'dgc':
        from grace_amd.torch.compressor.dgc import DgcCompressor
        compressor = DgcCompressor(params.get('compress_ratio', 0.3))
    elif comp == 'efsignsgd':
        from grace_amd.torch.compressor.efsignsgd import EFSignSGDCompressor
        compressor = EFSignSGDCompressor(params.get('lr', 0.1))
    elif comp == 'fp16':
        from grace_amd.torch.compressor.fp16 import FP16Compressor
        compressor = FP16Compressor()
    elif comp == 'natural':
        from grace_amd.torch.compressor.natural import NaturalCompressor
        compressor = NaturalCompressor()
    elif comp == 'none':
        from grace_amd.torch.compressor.none import NoneCompressor
        compressor = NoneCompressor()
    elif comp == 'onebit':
        from grace_amd.torch.compressor.onebit import OneBitCompressor
        compressor = OneBitCompressor()
    elif comp == 'powersgd':
        from grace_amd.torch.compressor.powersgd import PowerSGDCompressor
        compressor = PowerSGDCompressor()
    elif comp == 'qsgd':
        from grace_amd.torch.compressor.qsgd import QSGDCompressor
        compressor = QSGDCompressor(params.get('quantum_num', 127))
    elif comp == 'randomk':
        from grace_amd.torch.compressor.randomk import RandomKCompressor
        compressor = RandomKCompressor(params.get('compress_ratio', 0.3))
    elif comp == 'signsgd':
        from grace_amd.torch.compressor.signsgd import SignSGDCompressor
        compressor = SignSGDCompressor()
    elif comp == 'signum':
        from grace_amd.torch.compressor.signum import SignumCompressor
        compressor = SignumCompressor(params.get('momentum', 0.9))
    elif comp == 'terngrad':
        from grace_amd.torch.compressor.terngrad import TernGradCompressor
        compressor = TernGradCompressor()
    elif comp == 'threshold':
        from grace_amd.torch.compressor.threshold import ThresholdCompressor
        compressor = ThresholdCompressor(params.get('threshold', 0.01))
    elif comp == 'topk':
        from grace_amd.torch.compressor.topk import TopKCompressor
        compressor = TopKCompressor(params.get('compress_ratio', 0.3))
    else:
        raise NotImplementedError(comp)

    if mem == 'dgc':
        from grace_amd.torch.memory.dgc import DgcMemory
        memory = DgcMemory(params.get('momentum', 0.9), params.get('gradient_clipping', False))
    elif mem == 'none':
        from grace_amd.torch.memory.none import NoneMemory
        memory = NoneMemory()
    elif mem == 'powersgd':
        from grace_amd.torch.memory.powersgd import PowerSGDMemory
        memory = PowerSGDMemory(compressor.q_memory, params.get('compress_rank', 1))
    elif mem == 'residual':
        from grace_amd.torch.memory.residual import ResidualMemory
        memory = ResidualMemory()
    elif mem == 'efsignsgd':
        from grace_amd.torch.memory.efsignsgd import EFSignSGDMemory
        memory = EFSignSGDMemory(params.get('lr', 0.1))
    else:
        raise NotImplementedError(mem)

    if comm == 'allreduce':
        from grace_amd.torch.communicator.allreduce import Allreduce
        return Allreduce(compressor, memory, world_size)
    if comm == 'allgather':
        from grace_amd.torch.communicator.allgather import Allgather
        return Allgather(compressor, memory, world_size)
    if comm == 'broadcast':
        from grace_amd.torch.communicator.broadcast import Broadcast
        return Broadcast(compressor, memory, world_size)
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
