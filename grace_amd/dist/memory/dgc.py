"""DGC momentum-correction memory (grace_dl/dist/memory/dgc.py:6-39) on HIP kernels.

compensate: (optional clipping) r = momentum r + g, a = a + r, returns a (first step: r = a = g);
update: r = r * ~mask, a = a * ~mask with mask = |t| >= the compressor's final threshold.
The residual / accumulator buffers are owned by the memory and updated in place by compensate /
update; the world-1 fused step (DgcCompressor.fused_step) writes the new state into new buffers
and rebinds them, as the reference rebinds new tensors (the values are identical either way).  gradient_clipping=True implements the documented
intent -- clamp to sqrt(all_reduce(sum(g*g)) / world_size) -- where the reference itself raises a
TypeError (``dist.all_reduce`` returns None, memory/dgc.py:17-18).
"""
import torch
import torch.distributed as dist

from grace_amd import ops
from grace_amd.dist import Memory


class DgcMemory(Memory):
    def __init__(self, momentum, gradient_clipping, world_size):
        self.gradient_clipping = gradient_clipping
        self.momentum = momentum
        self.world_size = world_size
        self.gradients = {}
        self.residuals = {}

    def compensate(self, tensor, name):
        g = ops.dev_f32(tensor)
        if self.gradient_clipping:
            s = ops.sumsq(g)
            if dist.is_available() and dist.is_initialized():
                dist.all_reduce(s)
            g = ops.clip_by_sumsq(g, s, self.world_size)
        res = self.residuals.get(name)
        has = res is not None and res.numel() == g.numel()
        if not has:
            res = torch.empty_like(g)
            acc = torch.empty_like(g)
            self.residuals[name] = res
            self.gradients[name] = acc
        acc = self.gradients[name]
        ops.dgc_compensate(g, res, acc, has, self.momentum)
        return acc.view(tensor.shape)

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        _, meta, _ = ctx
        ops.dgc_mask_update(tensor.reshape(-1), self.residuals[name], self.gradients[name], meta)
