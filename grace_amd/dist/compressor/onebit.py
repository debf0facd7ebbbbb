"""One-bit quantisation (grace_dl/dist/compressor/onebit.py:6-31): payload (mask0 u8 = x<0,
mean0, mean1).  Decode uses the fixed semantics of grace_dl/torch/compressor/onebit.py:29 by
default; ``compat_uint8_not=True`` reproduces the dist flavour's uint8 ``~`` (254/255 weights)."""
from grace_amd import ops
from grace_amd.dist import Compressor


class OneBitCompressor(Compressor):

    def __init__(self, compat_uint8_not=False):
        super().__init__()
        self.compat_uint8_not = compat_uint8_not

    def compress(self, tensor, name):
        mask0, means = ops.onebit_encode(tensor)
        return (mask0, means[0:1], means[1:2]), tensor.size()

    def decompress(self, tensor_compressed, shape):
        mask0, mean0, mean1 = tensor_compressed
        return ops.onebit_decode(mask0, mean0, mean1, quirk=self.compat_uint8_not).view(shape)
