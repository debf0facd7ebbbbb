"""signSGD (grace_dl/dist/compressor/signsgd.py:6-30): u8 codeword (x >= 0), decode 2c-1,
majority-vote aggregate.  average=False as in the reference."""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class SignSGDCompressor(Compressor):

    def __init__(self):
        super().__init__(average=False)

    def compress(self, tensor, name):
        return [ops.sign_encode(tensor)], tensor.size()

    def decompress(self, tensors, shape):
        sign_encode, = tensors
        return ops.sign_decode(sign_encode).view(shape)

    def aggregate(self, tensors):
        """sum >= 0 -> +1 else -1 (signsgd.py:25-30)."""
        if not tensors[0].is_cuda:
            return super().aggregate(tensors)
        s = ops.sum_rank_order(tensors)
        codes = ops.sign_encode(s)
        return ops.sign_decode(codes).view(tensors[0].shape)

    def decode_aggregate_gathered(self, gathered, shape, world_size):
        codes, = gathered
        if not codes.is_cuda:
            return None
        n = shape.numel()
        return ops.sign_majority(codes, world_size, n).view(shape)

    def fused_step(self, communicator, tensor, name):
        from grace_amd.dist.communicator.allgather import Allgather
        from grace_amd.dist.memory.none import NoneMemory
        if (isinstance(communicator, Allgather) and type(communicator.memory) is NoneMemory
                and int(communicator.world_size) == 1 and isinstance(tensor, torch.Tensor)
                and tensor.is_cuda and tensor.dtype == torch.float32):
            _, out = ops.sign_step_w1(tensor)
            return out.view(tensor.shape)
        return None
