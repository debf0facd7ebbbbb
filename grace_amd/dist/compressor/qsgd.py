"""QSGD (grace_dl/dist/compressor/qsgd.py:5-77) on the HIP quantiser (grace_amd/csrc/quant.hip).

Payload (codes, bucket_norms): int8 codes for quantum_num < 128, fp16 otherwise (qsgd.py:37);
norms f32[ceil(n / bucket_size)].  ``rng='device'`` (default) draws the stochastic-rounding
uniforms on the GPU (counter-based, keyed by rank/name/step); ``rng='torch_cpu'`` draws them from
torch's global CPU generator exactly as the reference does (``torch.empty_like(x).uniform_()``,
qsgd.py:31) and copies them over, for bit-for-bit parity with the CPU reference.
``QSGDCompressor_CUDA`` follows the reference's qsgd_cuda extension semantics (f64 norms over finite
elements, one division for q / norm, NaN/Inf -> -128 -> NaN; qsgd_cuda.cu:320-408).
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class _QSGDBase(Compressor):
    variant = 0

    def __init__(self, quantum_num, bucket_size=128, rng="device"):
        super().__init__()
        self.quantum_num = quantum_num
        self.bucket_size = bucket_size
        self.rng = rng
        self._step = 0

    def _uniforms(self, n, name, device):
        self._step += 1
        if self.rng == "torch_cpu":
            return torch.empty(n).uniform_().to(device), 0
        return None, ops.step_seed("qsgd", ops.rank_of_process(), name, self._step)

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        u, seed = self._uniforms(flat.numel(), name, flat.device)
        codes, norms = ops.qsgd_compress(flat, self.quantum_num, self.bucket_size, variant=self.variant,
                                         u=u, seed=seed)
        return (codes, norms), tensor.size()

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(QSGD, NoneMemory).step at bucket 128 in one pass (grace_qsgd_step_w1):
        the codes compress() would draw (same generator step), decoded as (0 + d) / 1 and never
        stored -- bit-identical to compress + Allgather decode."""
        if not (ops.w1_elementwise_ok(communicator, tensor) and ops.qsgd_step_w1_ok([tensor.numel()], self.bucket_size)):
            return None
        u, seed = self._uniforms(tensor.numel(), name, tensor.device)
        return ops.qsgd_step_w1(tensor.view(-1), self.quantum_num, variant=self.variant, u=u, seed=seed).view(tensor.shape)

    def decompress(self, tensor_compressed, ctx):
        codes, norms = tensor_compressed
        shape = ctx
        return ops.qsgd_decompress(codes, norms, self.quantum_num, self.bucket_size, shape.numel(),
                                   variant=self.variant).view(shape)

    def decode_aggregate_gathered(self, gathered, shape, world_size):
        """Decode + rank-ordered aggregate + average of W payloads in one pass."""
        codes, norms = gathered
        if not codes.is_cuda:
            return None
        return ops.qsgd_decompress(codes, norms, self.quantum_num, self.bucket_size, shape.numel(),
                                   variant=self.variant, world=world_size, aggregate=True,
                                   divisor=world_size if self.average else 1.0).view(shape)


    # AllToAll hooks (grace_amd/dist/communicator/all_to_all.py): one launch per phase
    def a2a_decode_sum(self, gathered, chunk, world_size):
        codes, norms = gathered
        if not codes.is_cuda:
            return None
        return ops.qsgd_decompress(codes, norms, self.quantum_num, self.bucket_size, chunk, variant=self.variant,
                                   world=world_size, aggregate=True)

    def a2a_decode_concat(self, gathered, chunk, world_size):
        codes, norms = gathered
        if not codes.is_cuda:
            return None
        return ops.qsgd_decompress(codes, norms, self.quantum_num, self.bucket_size, world_size * chunk,
                                   variant=self.variant)


class QSGDCompressor(_QSGDBase):
    variant = 0


class QSGDCompressor_CUDA(_QSGDBase):
    variant = 1
