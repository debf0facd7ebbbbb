from grace_amd.dist import Compressor


class NoneCompressor(Compressor):
    """Default no-op compression (grace_dl/dist/compressor/none.py:4-12)."""

    def compress(self, tensor, name):
        return [tensor], None

    def decompress(self, tensors, ctx):
        tensor, = tensors
        return tensor
