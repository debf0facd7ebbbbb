"""Top-k, Horovod flavour (grace_dl/torch/compressor/topk.py:6-36) on the HIP top-k engine.

Differs from the dist copy: the payload keeps torch.topk's int64 indices and ctx is
``(numel, shape)``.  Same exact selector as grace_amd.dist (larger |x| first, lower index first
among ties; torch.topk(sorted=False) returns the same set modulo ties at the k-th magnitude)."""
from grace_amd import ops
from grace_amd.dist import Compressor


class TopKCompressor(Compressor):

    def __init__(self, compress_ratio):
        super().__init__()
        self.compress_ratio = compress_ratio

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        k = ops.ratio_k(flat.numel(), self.compress_ratio)
        _, vals, idx32 = ops.topk_compress(flat, k)
        return [vals, ops.widen_i32(idx32)], (tensor.numel(), tensor.size())

    def decompress(self, tensors, ctx):
        numel, shape = ctx
        values, indices = tensors
        return ops.sparse_decode(values, indices, numel).view(shape)
