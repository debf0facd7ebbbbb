"""EF-signSGD (grace_dl/dist/compressor/efsignsgd.py:6-33): payload (mean|x| f32[1], u8 signs),
decode mean * (2s - 1), aggregate sum / lr."""
from grace_amd import ops
from grace_amd.dist import Compressor


class EFSignSGDCompressor(Compressor):

    def __init__(self, lr):
        super().__init__(average=False)
        self.learning_rate = lr

    def compress(self, tensor, name):
        mean = ops.abs_mean(tensor)
        return (mean, ops.sign_encode(tensor)), tensor.size()

    def decompress(self, tensor_compressed, shape):
        mean, sign_encode = tensor_compressed
        return ops.sign_decode(sign_encode, scale=mean).view(shape)

    def aggregate(self, tensors):
        if not tensors[0].is_cuda:
            return sum(tensors) / self.learning_rate
        return ops.div_scalar(ops.sum_rank_order(tensors), self.learning_rate).view(tensors[0].shape)
