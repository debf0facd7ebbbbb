"""Deep Gradient Compression (grace_dl/dist/compressor/dgc.py:12-50) on the HIP DGC engine
(grace_amd/csrc/dgc.hip).

Payload = [values f32[m], indices int64[m]] with m data-dependent (tensors_size_are_same=False,
so Allgather exchanges sizes first), indices ascending like torch.where.  The 1 % sample is
uniform with replacement: ``rng='torch_cpu'`` draws it from torch's global CPU generator exactly
like the reference (uniform_(0, numel).long(); parity mode), ``rng='device'`` (default) uses the
counter-based device generator.  The threshold adjustment loop (<= 10 rounds of x1.3 / x0.7) is
replayed on exact counts from one histogram pass instead of one full pass per round.
ctx = (shape, meta, numel): ``meta`` (16 bytes on the device) carries the final threshold that
DgcMemory.update turns back into the mask (the reference carries the n-element bool mask).
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class DgcCompressor(Compressor):

    def __init__(self, compress_ratio, rng="device"):
        super().__init__(tensors_size_are_same=False)
        self.compress_ratio = compress_ratio
        self.rng = rng
        self._step = 0

    def _sampling(self, t, name):
        """(sample indices, seed) of this call: the reference's CPU uniform_ stream in parity mode,
        else the device generator keyed by (name, step)."""
        numel = t.numel()
        if self.rng == "torch_cpu":
            ns = max(1, int(numel * 0.01))
            cpu = torch.empty([ns]).uniform_(0, numel).type(torch.long)
            if ns and int(cpu.max()) >= numel:       # the reference would raise IndexError here
                raise IndexError(f"DGC sample index {int(cpu.max())} out of range for {numel} elements")
            return cpu.to(t.device), 0
        self._step += 1
        return None, ops.step_seed("dgc", name, self._step)

    def compress(self, tensor, name):
        shape = tensor.size()
        t = ops.dev_f32(tensor)
        sidx, seed = self._sampling(t, name)
        vals, idx, meta = ops.dgc_compress(t, self.compress_ratio, sample_idx=sidx, seed=seed)
        return (vals, idx), (shape, meta, t.numel())

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(DgcCompressor, DgcMemory).step: compensate, the threshold, then ONE
        pass for DgcMemory.update and (0 + decompress) / 1 -- the same values as the four calls,
        without materialising the payload or reading its size on the host."""
        from grace_amd.dist.communicator.allgather import Allgather
        from grace_amd.dist.memory.dgc import DgcMemory
        mem = communicator.memory
        if not (type(communicator) is Allgather and type(mem) is DgcMemory and int(communicator.world_size) == 1
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        t = ops.dev_f32(mem.compensate(tensor, name))
        sidx, seed = self._sampling(t, name)
        ws = ops.dgc_select(t, self.compress_ratio, sample_idx=sidx, seed=seed)
        out = ops.dgc_step_w1(t, mem.residuals[name], mem.gradients[name], ws)
        return out.view(tensor.shape)

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        shape, _, numel = ctx
        return ops.sparse_decode(values, indices, numel).view(shape)
