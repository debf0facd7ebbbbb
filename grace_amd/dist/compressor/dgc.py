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

    def compress(self, tensor, name):
        shape = tensor.size()
        t = ops.dev_f32(tensor)
        numel = t.numel()
        sidx = None
        seed = 0
        if self.rng == "torch_cpu":
            ns = max(1, int(numel * 0.01))
            cpu = torch.empty([ns]).uniform_(0, numel).type(torch.long)
            if ns and int(cpu.max()) >= numel:       # the reference would raise IndexError here
                raise IndexError(f"DGC sample index {int(cpu.max())} out of range for {numel} elements")
            sidx = cpu.to(t.device)
        else:
            self._step += 1
            seed = ops.step_seed("dgc", name, self._step)
        vals, idx, meta = ops.dgc_compress(t, self.compress_ratio, sample_idx=sidx, seed=seed)
        return (vals, idx), (shape, meta, numel)

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        shape, _, numel = ctx
        return ops.sparse_decode(values, indices, numel).view(shape)
