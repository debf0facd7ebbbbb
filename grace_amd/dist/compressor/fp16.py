"""FP16 cast compression (grace_dl/dist/compressor/fp16.py:6-22) on HIP cast kernels."""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class FP16Compressor(Compressor):
    """Compress all floating point gradients to 16-bit."""

    def compress(self, tensor, name):
        dtype = tensor.dtype
        if dtype == torch.float32:
            return [ops.fp16_compress(tensor).view(tensor.shape)], dtype
        if dtype.is_floating_point and tensor.is_cuda:
            raise TypeError(f"grace_amd FP16Compressor supports float32 gradients, got {dtype}")
        return [tensor], dtype

    def decompress(self, tensors, dtype):
        tensor_decompressed, = tensors
        if dtype == torch.float32:
            return ops.fp16_decompress(tensor_decompressed).view(tensor_decompressed.shape)
        return tensor_decompressed
