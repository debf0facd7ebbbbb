"""EF-signSGD memory (grace_dl/dist/memory/efsignsgd.py:4-19): t = r + lr * g, r' = t - decode."""
from grace_amd import ops
from grace_amd.dist import Memory


class EFSignSGDMemory(Memory):
    def __init__(self, lr):
        self.residuals = {}
        self.learning_rate = lr

    def compensate(self, tensor, name):
        if name in self.residuals:
            return ops.axpby(self.residuals[name], tensor, 1.0, self.learning_rate).view(tensor.shape)
        return tensor

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        tensor_decompressed = compressor.decompress(tensor_compressed, ctx)
        self.residuals[name] = ops.sub(tensor, tensor_decompressed)
