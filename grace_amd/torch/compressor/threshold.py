"""Threshold sparsification, Horovod flavour (grace_dl/torch/compressor/threshold.py:6-27).

Differs from the dist copy: ``|x| > threshold`` (strict, no min(threshold, max(x)) rule), int64
indices and ctx ``(shape, numel)``.  Ascending index order (torch.where), variable size."""
from grace_amd import ops
from grace_amd.dist import Compressor


class ThresholdCompressor(Compressor):

    def __init__(self, threshold):
        super().__init__(tensors_size_are_same=False)
        self.threshold = threshold

    def compress(self, tensor, name):
        shape = tensor.size()
        values, indices = ops.threshold_compress_strict(tensor, self.threshold)
        return [values, indices], (shape, tensor.numel())

    def decompress(self, tensor_compressed, ctx):
        shape, numel = ctx
        values, indices = tensor_compressed
        return ops.sparse_decode(values, indices, numel).view(shape)
