"""QSGD, Horovod flavour (grace_dl/torch/compressor/qsgd.py:7-39) on grace_qsgd_global_compress.

Unlike the dist copy (per-128 bucket norms), the torch copy quantises against ONE norm over the
whole tensor: ``norm = tensor.norm()``; ``level = q / norm * |x|`` (torch's ``__rdiv__``:
reciprocal(norm) * q); stochastic rounding with ``uniform_()``; ``int16`` then int8 (q < 128) or
fp16.  Payload (codes[n], norm f32[1]); decompress ``norm / q * code``.  ``rng='torch_cpu'`` draws the
uniforms from torch's CPU generator exactly as the reference; ``'device'`` uses the counter-based
device generator keyed by (rank, name, step).
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class QSGDCompressor(Compressor):

    def __init__(self, quantum_num, rng="device"):
        super().__init__()
        self.quantum_num = quantum_num
        self.rng = rng
        self._step = 0

    def compress(self, tensor, name):
        shape = tensor.size()
        flat = ops.dev_f32(tensor)
        self._step += 1
        if self.rng == "torch_cpu":
            u, seed = torch.empty(flat.numel()).uniform_().to(flat.device), 0
        else:
            u, seed = None, ops.step_seed("qsgd-global", ops.rank_of_process(), name, self._step)
        codes, norm = ops.qsgd_global_compress(flat, self.quantum_num, u=u, seed=seed)
        return (codes, norm), shape

    def decompress(self, tensor_compressed, shape):
        codes, norm = tensor_compressed
        return ops.qsgd_global_decompress(codes, norm, self.quantum_num, shape.numel()).view(shape)
