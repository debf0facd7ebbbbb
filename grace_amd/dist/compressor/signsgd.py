"""signSGD (grace_dl/dist/compressor/signsgd.py:6-30): u8 codeword (x >= 0), decode 2c-1,
majority-vote aggregate.  average=False as in the reference.

``wire='bits'`` sends the same codewords packed 1 bit per element (8x fewer bytes on the wire;
grace_amd/csrc/wire.hip), and the Allgather majority vote runs on the packed payloads directly.
The default ``wire='u8'`` is the reference's payload."""
import torch

from grace_amd import ops
from grace_amd.dist.communicator.allgather import Allgather
from grace_amd.dist.memory.none import NoneMemory
from grace_amd.dist import Compressor


class SignSGDCompressor(Compressor):

    def __init__(self, wire="u8"):
        super().__init__(average=False)
        if wire not in ("u8", "bits"):
            raise ValueError("wire must be 'u8' or 'bits'")
        self.wire = wire

    def compress(self, tensor, name):
        codes = ops.sign_encode(tensor)
        if self.wire == "bits":
            return [ops.pack_bits(codes)], tensor.size()
        return [codes], tensor.size()

    def decompress(self, tensors, shape):
        sign_encode, = tensors
        if self.wire == "bits":
            sign_encode = ops.unpack_bits(sign_encode, shape.numel())
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
        if self.wire == "bits":
            return ops.sign_majority_bits(codes, world_size, n).view(shape)
        return ops.sign_majority(codes, world_size, n).view(shape)

    def fused_step(self, communicator, tensor, name):
        if (isinstance(communicator, Allgather) and type(communicator.memory) is NoneMemory
                and int(communicator.world_size) == 1 and isinstance(tensor, torch.Tensor)
                and tensor.is_cuda and tensor.dtype == torch.float32):
            _, out = ops.sign_step_w1(tensor, want_codes=False, reuse_out=True)
            return out if out.shape == tensor.shape else out.view(tensor.shape)
        return None
