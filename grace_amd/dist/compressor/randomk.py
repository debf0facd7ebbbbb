"""Random-k sparsification (grace_dl/dist/compressor/randomk.py:6-41).

Seed h = sum(bytes(name)) + global_step, global_step one counter per compressor instance (so all
ranks draw the same indices), k = max(1, int(numel * ratio)) indices WITH replacement, payload
[values f32[k]], ctx (indices, numel, shape).  Like the reference, compress reseeds torch's global
generator with h.  ``rng='device'`` (default) draws the indices on the GPU from a counter-based
generator keyed by h (deterministic, identical on every rank, not bit-equal to torch's stream);
``rng='torch_cpu'`` draws them with torch's CPU generator exactly as the reference does on CPU.
"""
import torch

from grace_amd import ops
from grace_amd.dist import Compressor


class RandomKCompressor(Compressor):

    def __init__(self, compress_ratio, rng="device", recycle_output=True):
        super().__init__()
        self.global_step = 0
        self.compress_ratio = compress_ratio
        self.rng = rng
        self.recycle_output = recycle_output   # world-1 step: reuse a dropped, unmodified result
        self._recycler = ops.OutputRecycler()
        self._grp = {}

    def _indices(self, flat, name):
        """randomk.py:26-30: the seed h, the global generator reseeded with it, k indices drawn with
        replacement (torch's CPU stream in parity mode, else the device generator keyed by h)."""
        numel = flat.numel()
        h = sum(bytes(name, encoding='utf8'), self.global_step)
        self.global_step += 1
        torch.manual_seed(h)
        k = ops.ratio_k(numel, self.compress_ratio)
        if self.rng == "torch_cpu":
            return torch.randint(numel, [k]).to(flat.device)
        return ops.randomk_indices(h, numel, k, flat.device)

    def fused_step(self, communicator, tensor, name):
        """World-1 Allgather(RandomK, ResidualMemory).step: the indices grouped by chunk, then one
        streaming pass for r' and out (grace_randomk_step_w1_dense; no payload at world 1) -- the
        same values as compensate + compress + update + send_receive."""
        from grace_amd.dist.communicator.allgather import Allgather
        from grace_amd.dist.memory.residual import ResidualMemory
        mem = communicator.memory
        if not (type(communicator) is Allgather and type(mem) is ResidualMemory and int(communicator.world_size) == 1
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        g = ops.dev_f32(tensor)
        res = mem.residuals.get(name)
        has = res is not None and res.numel() == g.numel() and res.device == g.device
        if not has:
            res = torch.empty_like(g)
        indices = self._indices(g, name)
        if g.numel() <= ops.SORT_PAYLOAD_MAX_N:
            if self.recycle_output:
                # the dropped, unmodified previous result of this name comes back (ops.OutputRecycler)
                # with the grouping of its indices: only those positions are cleared and only the
                # drawn ones written; the two grouping buffers of a name alternate
                out, prev = self._recycler.take(name, g)
                key = (g.numel(), indices.numel(), g.device)
                bufs = self._grp.get(name)
                if bufs is None or bufs[0] != key:
                    nb = ops.randomk_group_bytes(g.numel(), indices.numel())
                    bufs = self._grp[name] = (key, [torch.empty(nb, dtype=torch.uint8, device=g.device) for _ in range(2)])
                    prev = None
                grp = bufs[1][1] if prev is bufs[1][0] else bufs[1][0]
                out = ops.randomk_step_w1_dense(g, res, has, mem.beta, mem.gamma, indices, out=out, grp=grp,
                                                prev_grp=prev)
                self._recycler.keep(name, out, grp)
            else:
                out = ops.randomk_step_w1_dense(g, res, has, mem.beta, mem.gamma, indices)
        else:
            _, out = ops.randomk_step_w1(g, res, has, mem.beta, mem.gamma, indices)
        mem.residuals[name] = res
        return out.view(tensor.shape)

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        indices = self._indices(flat, name)
        numel = flat.numel()
        values = ops.gather(flat, indices)
        ctx = indices, numel, tensor.size()
        return [values], ctx

    def decompress(self, tensors, ctx):
        indices, numel, shape = ctx
        values, = tensors
        return ops.sparse_decode(values, indices, numel).view(shape)
