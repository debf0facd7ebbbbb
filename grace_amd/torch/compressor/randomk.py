"""Random-k, Horovod flavour (grace_dl/torch/compressor/randomk.py:6-41).

Differs from the dist copy: the k indices are ``randperm(numel)[:k]`` -- WITHOUT replacement.
Seed ``h = sum(bytes(name)) + global_step`` and ``torch.manual_seed(h)`` as the reference (so every
rank draws the same indices).  ``rng='device'`` (default): k distinct indices from a keyed
permutation of [0, numel) on the GPU (grace_randomk_perm_indices); ``rng='torch_cpu'``: torch's CPU
randperm exactly as the reference (bit-parity mode).  Payload [values f32[k]], ctx
(indices int64, numel, shape)."""
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
            indices = torch.randperm(numel)[:k].to(flat.device)
        else:
            indices = ops.randomk_perm_indices(h, numel, k, flat.device)
        values = ops.gather(flat, indices)
        return [values], (indices, numel, tensor.size())

    def decompress(self, tensors, ctx):
        indices, numel, shape = ctx
        values, = tensors
        return ops.sparse_decode(values, indices, numel).view(shape)
