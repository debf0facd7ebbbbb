"""FP16 cast compression (grace_dl/dist/compressor/fp16.py:6-22) on HIP cast kernels.

ctx carries (dtype, shape) instead of the reference's dtype alone, so the Allgather fast path can
restore the shape after decoding the flat gathered payloads (callers treat ctx as opaque)."""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class FP16Compressor(Compressor):
    """Compress all floating point gradients to 16-bit."""

    def compress(self, tensor, name):
        dtype = tensor.dtype
        if dtype == torch.float32:
            return [ops.fp16_compress(tensor).view(tensor.shape)], (dtype, tensor.shape)
        if dtype.is_floating_point and tensor.is_cuda:
            raise TypeError(f"grace_amd FP16Compressor supports float32 gradients, got {dtype}")
        return [tensor], (dtype, tensor.shape)

    def decompress(self, tensors, ctx):
        tensor_decompressed, = tensors
        dtype = ctx[0] if isinstance(ctx, tuple) else ctx
        if dtype == torch.float32:
            return ops.fp16_decompress(tensor_decompressed).view(tensor_decompressed.shape)
        return tensor_decompressed

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(FP16, NoneMemory).step as ONE pass (grace_cast_step_w1):
        (0 + f32(f16(x))) / 1, the f16 payload never stored."""
        if not ops.w1_elementwise_ok(communicator, tensor):
            return None
        return ops.cast_step_w1(tensor, 3, 0)

    def decode_aggregate_gathered(self, gathered, ctx, world_size):
        """Allgather (allgather.py:40-45): the W gathered f16 payloads decoded, summed in rank order
        from 0 and divided by W (if averaging) in one native pass."""
        h, = gathered
        dtype, shape = ctx
        if dtype != torch.float32 or not h.is_cuda or h.dtype != torch.float16:
            return None
        n = h.numel() // world_size
        return ops.fp16_decompress_aggregate(h, n, world_size, divisor=world_size if self.average else 1.0).view(shape)
