"""PowerSGD, Horovod flavour (grace_dl/torch/compressor/powersgd.py:21-58) on the HIP kernels.

Differs from the dist copy: no rank / use_memory / world_size arguments -- q is ALWAYS taken from
``q_memory[name]`` (drawn by PowerSGDMemory.compensate, whose compress_rank sets the rank) and
orthogonalised in place; P and Q are averaged over the ranks (Horovod's ``allreduce_`` averages by
default); ``q_memory[name] = Q`` afterwards.  Parity unpinned: the reference module imports horovod,
which is absent, so it is checked against the oracle's restatement (tests/test_gpu_torch_flavour.py).
"""
import torch.distributed as dist

from grace_amd import ops
from grace_amd.dist import Compressor


def orthogonalize(matrix):
    return ops.orthogonalize_(matrix)


def _allreduce_average(t):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
        return ops.div_scalar(t, dist.get_world_size()).view(t.shape)
    return t


class PowerSGDCompressor(Compressor):

    def __init__(self):
        super().__init__()
        self.q_memory = {}

    def compress(self, tensor, name):
        if tensor.dim() == 1:
            return [tensor], None
        shape = tensor.size()
        matrix = ops.dev_f32(tensor).view(shape[0], -1)
        q = self.q_memory[name]
        orthogonalize(q)
        p = _allreduce_average(ops.powersgd_p(matrix, q))
        orthogonalize(p)
        q = _allreduce_average(ops.powersgd_qt(matrix, p))
        self.q_memory[name] = q
        return [], (p, q, shape)

    def decompress(self, tensors, ctx):
        if ctx is None:
            tensor, = tensors
            return tensor
        p, q, tensor_shape = ctx
        out, _ = ops.powersgd_outer(p, q)
        return out.view(tensor_shape)
