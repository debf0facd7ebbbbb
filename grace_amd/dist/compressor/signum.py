"""Signum (grace_dl/dist/compressor/signum.py:6-37): per-name momentum m = (1-b) g + b m, then
the signSGD codeword; momentum buffers live on the device."""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class SignumCompressor(Compressor):

    def __init__(self, momentum):
        super().__init__(average=False)
        self.momentum = momentum
        self.momentums = {}

    def compress(self, tensor, name):
        g = ops.dev_f32(tensor)
        buf = self.momentums.get(name)
        has_prev = buf is not None and buf.numel() == g.numel()
        if not has_prev:
            buf = torch.empty_like(g)
        codes = ops.signum_encode(g, buf, has_prev, self.momentum)
        self.momentums[name] = buf
        return [codes], tensor.size()

    def decompress(self, tensors, shape):
        sign_encode, = tensors
        return ops.sign_decode(sign_encode).view(shape)

    def aggregate(self, tensors):
        if not tensors[0].is_cuda:
            return super().aggregate(tensors)
        s = ops.sum_rank_order(tensors)
        return ops.sign_decode(ops.sign_encode(s)).view(tensors[0].shape)

    def decode_aggregate_gathered(self, gathered, shape, world_size):
        codes, = gathered
        if not codes.is_cuda:
            return None
        return ops.sign_majority(codes, world_size, shape.numel()).view(shape)
