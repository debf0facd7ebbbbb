"""Natural compression.  ``NaturalCompressor`` reproduces the cupy codec bit-for-bit
(grace_dl/dist/compressor/natural.py:8-40: exponent rounded up when the mantissa exceeds a random
int in [0, 2^23-1), clipped to [18, 145], u8 = sign | (E - 18)); ``NaturalCompressor_CUDA`` the
cnat_cuda extension's LUT encoding (cnat_cuda.cu:68-134), whose codes are offset by one exponent
step from the cupy ones — the two wire formats are not interchangeable, as in the reference.
``rng='torch_cpu'`` injects a host-drawn random stream (tests); default draws on the device.
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class NaturalCompressor(Compressor):
    flavour = 0

    def __init__(self, rng="device"):
        super().__init__()
        self.rng = rng
        self._step = 0

    def _encode(self, flat, name):
        self._step += 1
        if self.rng == "torch_cpu":
            ri = torch.randint(0, 0x7FFFFF, (flat.numel(),), dtype=torch.int32).to(flat.device)
            return ops.natural_compress(flat, rand_int=ri)
        return ops.natural_compress(flat, seed=ops.step_seed("natural", ops.rank_of_process(), name, self._step))

    def compress(self, tensor, name):
        return [self._encode(ops.dev_f32(tensor), name)], tensor.size()

    def _w1_mode(self):
        return 0 if self.rng == "device" else None

    def _w1_seed(self, name):
        return ops.step_seed("natural", ops.rank_of_process(), name, self._step)

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(Natural, NoneMemory).step as ONE pass (grace_cast_step_w1): the same
        codes as compress() on the device generator, decoded as (0 + d) / 1, never stored."""
        mode = self._w1_mode()
        if mode is None or not ops.w1_elementwise_ok(communicator, tensor):
            return None
        self._step += 1
        return ops.cast_step_w1(tensor, mode, self._w1_seed(name))

    def decompress(self, tensor_compressed, shape):
        codes, = tensor_compressed
        return ops.natural_decompress(codes, shape.numel(), self.flavour).view(shape)

    def decode_aggregate_gathered(self, gathered, shape, world_size):
        codes, = gathered
        if not codes.is_cuda:
            return None
        return ops.natural_decompress(codes, shape.numel(), self.flavour, world=world_size, aggregate=True,
                                      divisor=world_size if self.average else 1.0).view(shape)


    # AllToAll hooks (grace_amd/dist/communicator/all_to_all.py): one launch per phase
    def a2a_decode_sum(self, gathered, chunk, world_size):
        codes, = gathered
        if not codes.is_cuda:
            return None
        return ops.natural_decompress(codes, chunk, self.flavour, world=world_size, aggregate=True)

    def a2a_decode_concat(self, gathered, chunk, world_size):
        codes, = gathered
        if not codes.is_cuda:
            return None
        return ops.natural_decompress(codes, world_size * chunk, self.flavour)


class NaturalCompressor_CUDA(NaturalCompressor):
    flavour = 1

    def _w1_mode(self):
        return {"device": 1, "deterministic": 2}.get(self.rng)

    def _w1_seed(self, name):
        return ops.step_seed("cnat", ops.rank_of_process(), name, self._step)

    def _encode(self, flat, name):
        self._step += 1
        if self.rng == "torch_cpu":
            return ops.cnat_compress(flat, rand=torch.rand(flat.numel()).to(flat.device))
        if self.rng == "deterministic":
            return ops.cnat_compress(flat, deterministic=True)
        return ops.cnat_compress(flat, seed=ops.step_seed("cnat", ops.rank_of_process(), name, self._step))
