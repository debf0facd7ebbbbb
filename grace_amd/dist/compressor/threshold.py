"""Threshold sparsification (grace_dl/dist/compressor/threshold.py:6-27): every element with
|x| >= min(threshold, max(x)) (signed max, as the reference), ascending index order, payload
[values f32[m], indices int32[m]] with m data-dependent (tensors_size_are_same=False)."""
from grace_amd import ops
from grace_amd.dist import Compressor


class ThresholdCompressor(Compressor):

    def __init__(self, threshold):
        super().__init__(tensors_size_are_same=False)
        self.threshold = threshold

    def compress(self, tensor, name):
        values, indices = ops.threshold_compress(tensor, self.threshold)
        return [values, indices], tensor.size()

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        return ops.sparse_decode(values, indices, ctx.numel()).view(ctx)

    def decode_aggregate_variable(self, gathered, sizes, ctx, world_size):
        """Variable-size Allgather: rank-ordered scatter-add of the W padded payloads."""
        vals, idx = gathered
        if not vals.is_cuda:
            return None
        stride = vals.numel() // world_size
        counts = [int(sizes[r][0]) for r in range(world_size)]
        out = ops.sparse_aggregate(vals, idx, stride, counts, world_size, ctx.numel(),
                                   world_size if self.average else 1)
        return out.view(ctx)
