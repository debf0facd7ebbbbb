"""TernGrad (grace_dl/dist/compressor/terngrad.py:5-30) on the HIP quantiser.

Payload (codes int8[n] in {-1,0,1}, scalar f32[1]).  The std / max reductions run in f64 on the
device (the reference's f32 CPU reduction order is not reproducible on a GPU; the scalar agrees
within a few ulp and codewords are bit-exact given the same clamp bound and uniforms, see
tests/test_gpu_quant.py).  ``rng`` as for QSGD.
``wire='2bit'`` sends the codes as code + 1 in the 2-bit byte layout of
grace_dl/tensorflow/compressor/packing.py (4x fewer bytes); the default ``wire='int8'`` is the
reference's payload.
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class TernGradCompressor(Compressor):

    def __init__(self, rng="device", wire="int8"):
        super().__init__()
        if wire not in ("int8", "2bit"):
            raise ValueError("wire must be 'int8' or '2bit'")
        self.rng = rng
        self.wire = wire
        self._step = 0

    def _uniforms(self, n, name, device):
        self._step += 1
        if self.rng == "torch_cpu":
            return torch.empty(n).uniform_(0, 1).to(device), 0
        return None, ops.step_seed("terngrad", ops.rank_of_process(), name, self._step)

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        u, seed = self._uniforms(flat.numel(), name, flat.device)
        codes, scalar = ops.terngrad_compress(flat, u=u, seed=seed)
        if self.wire == "2bit":
            codes = ops.tern_pack(codes)
        return (codes, scalar), tensor.size()

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(TernGrad, NoneMemory).step: statistics pass + one pass writing
        0 + code * scalar (grace_terngrad_step_w1), the codes compress() would draw never stored --
        bit-identical to compress + Allgather decode (the wire format does not matter at W=1)."""
        if not ops.w1_elementwise_ok(communicator, tensor):
            return None
        u, seed = self._uniforms(tensor.numel(), name, tensor.device)
        return ops.terngrad_step_w1(tensor.view(-1), u=u, seed=seed).view(tensor.shape)

    def decompress(self, tensor_compressed, ctx):
        codes, scalar = tensor_compressed
        if self.wire == "2bit":
            codes = ops.tern_unpack(codes, ctx.numel())
        return ops.terngrad_decompress(codes, scalar, ctx.numel()).view(ctx)

    def decode_aggregate_gathered(self, gathered, shape, world_size):
        codes, scalars = gathered
        if not codes.is_cuda or self.wire == "2bit":
            return None
        return ops.terngrad_decompress(codes, scalars, shape.numel(), world=world_size, aggregate=True,
                                       divisor=world_size if self.average else 1.0).view(shape)

    # AllToAll hooks (grace_amd/dist/communicator/all_to_all.py): one launch per phase
    def a2a_decode_sum(self, gathered, chunk, world_size):
        codes, scalars = gathered
        if not codes.is_cuda:
            return None
        return ops.terngrad_decompress(codes, scalars, chunk, world=world_size, aggregate=True)

    def a2a_decode_concat(self, gathered, chunk, world_size):
        codes, scalars = gathered
        if not codes.is_cuda:
            return None
        return ops.terngrad_decompress(codes, scalars, world_size * chunk, sizes=[chunk] * world_size)
