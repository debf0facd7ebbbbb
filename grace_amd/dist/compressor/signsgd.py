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
        if self.wire == "bits":
            return [ops.sign_encode_bits(tensor)], tensor.size()   # one pass, no u8 codes
        return [ops.sign_encode(tensor)], tensor.size()

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
        """World-1 Allgather(SignSGD, NoneMemory).step as ONE launch: sign encode -> decode ->
        majority of one = +-1 (signsgd.py:12-30).  A 4 MiB step is launch-bound (the kernel is
        ~1.5 us of HBM time), so this path keeps the host work to one checked ctypes launch."""
        if not (communicator.__class__ is Allgather and communicator.memory.__class__ is NoneMemory
                and communicator.world_size == 1):
            return None
        if not (tensor.__class__ is torch.Tensor and tensor.is_cuda and tensor.dtype == torch.float32
                and tensor.is_contiguous()):
            if not (isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
                return None
            _, out = ops.sign_step_w1(tensor, want_codes=False, reuse_out=True)
            return out.view(tensor.shape)
        out = ops.reusable_output("sign_w1", tensor.shape, torch.float32, tensor.device)
        ops.launch_sign_step_w1(tensor, out)
        return out
