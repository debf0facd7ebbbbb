"""Random-k sparsification (grace_dl/dist/compressor/randomk.py:6-41).

Seed h = sum(bytes(name)) + global_step, global_step one counter per compressor instance (so all
ranks draw the same indices), k = max(1, int(numel * ratio)) indices WITH replacement, payload
[values f32[k]], ctx (indices, numel, shape).  Like the reference, compress reseeds torch's global
generator with h.  ``rng='device'`` (default) draws the indices on the GPU from a counter-based
generator keyed by h (deterministic, identical on every rank, not bit-equal to torch's stream);
``rng='torch_cpu'`` draws them with torch's CPU generator exactly as the reference does on CPU.
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class RandomKCompressor(Compressor):

    def __init__(self, compress_ratio, rng="device"):
        super().__init__()
        self.global_step = 0
        self.compress_ratio = compress_ratio
        self.rng = rng

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        numel = flat.numel()
        h = sum(bytes(name, encoding='utf8'), self.global_step)
        self.global_step += 1
        torch.manual_seed(h)
        k = ops.ratio_k(numel, self.compress_ratio)
        if self.rng == "torch_cpu":
            indices = torch.randint(numel, [k]).to(flat.device)
        else:
            indices = ops.randomk_indices(h, numel, k, flat.device)
        values = ops.gather(flat, indices)
        ctx = indices, numel, tensor.size()
        return [values], ctx

    def decompress(self, tensors, ctx):
        indices, numel, shape = ctx
        values, = tensors
        return ops.sparse_decode(values, indices, numel).view(shape)
