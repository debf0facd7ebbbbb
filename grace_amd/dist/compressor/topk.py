"""Top-k sparsification (grace_dl/dist/compressor/topk.py:32-69) on the HIP top-k engine
(grace_amd/csrc/topk.hip).

Payload = [values f32[k], indices int32[k]] exactly as the reference (topk.py:41-42), ctx =
``tensor.size()``.  The selected set equals torch.topk(|x|, k, sorted=False)'s modulo ties at the
k-th magnitude; ours breaks ties by lower index.  ``kernel`` ('torch' | 'cupy' | 'rdxtopk_cuda',
topk.py:35-40) is accepted for compatibility: every value selects the same exact native selector.
"""
import torch
import torch.distributed as dist

from grace_amd import ops
from grace_amd.dist.communicator.allgather import Allgather
from grace_amd.dist.memory.none import NoneMemory
from grace_amd.dist.memory.residual import ResidualMemory
from grace_amd.dist import Compressor


class TopKCompressor(Compressor):

    def __init__(self, compress_ratio, kernel='torch', recycle_output=True, check_sync=False):
        super().__init__()
        self.compress_ratio = compress_ratio
        self.kernel = kernel
        # a run-out of the exact fallback's bounded waits (never expected) raises ops.TopKWaitError
        # at the next top-k call; check_sync=True waits for the device after every compress / step
        # and raises on the failing call itself
        self.check_sync = check_sync
        # world-1 step WITHOUT memory: reuse a dropped, unmodified previous result of the same name
        # and rewrite only its non-zeros (ops.OutputRecycler; A/B r04: 0.1356 -> 0.1272 ms).  The
        # residual step keeps the dense write: next to its g, r, r' streams the scattered writes
        # cost more than the 4 B per element they save (0.2137 -> 0.2294 ms, tools/ab_recycle.py);
        # recycle_output="always" turns it on there as well, False everywhere off.
        self.recycle_output = recycle_output
        self._recycler = ops.OutputRecycler()
        self.place_probes = {}   # name -> probe microseconds per (residual, output) pair tried (diagnostic)

    def compress(self, tensor, name):
        flat = ops.dev_f32(tensor)
        k = ops.ratio_k(flat.numel(), self.compress_ratio)
        _, vals, idx = ops.topk_compress(flat, k)
        if self.check_sync:
            ops.topk_check()
        return [vals, idx], tensor.size()

    def decompress(self, tensors, ctx):
        """Zeros with the values scattered back, reshaped to the original shape (topk.py:64-69)."""
        vals, idx = tensors
        return ops.sparse_decode(vals, idx, ctx.numel()).view(ctx)

    def decode_aggregate_gathered(self, gathered, ctx, world_size):
        """Allgather decode + aggregate + average of W same-size payloads in one rank-ordered
        scatter pass (allgather.py:40-45).  gathered = [vals f32[W*k], idx i32[W*k]]."""
        vals, idx = gathered
        if not vals.is_cuda:
            return None
        k = vals.numel() // world_size
        divisor = world_size if self.average else 1
        out = ops.sparse_aggregate(vals, idx, k, [k] * world_size, world_size, ctx.numel(), divisor)
        return out.view(ctx)

    def fused_step(self, communicator, tensor, name):
        """compensate -> compress -> update -> send_receive for (TopK, Residual, Allgather) at any world
        size, and for (TopK, NoneMemory, Allgather) at world 1."""
        out = self._fused_step(communicator, tensor, name)
        if out is not None and self.check_sync:
            ops.topk_check()
        return out

    def _fused_step(self, communicator, tensor, name):
        mem = communicator.memory
        if (isinstance(communicator, Allgather) and type(mem) is NoneMemory and int(communicator.world_size) == 1
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            # no memory, world 1: payload and (0 + d) / 1 from one read of the tensor
            g = ops.dev_f32(tensor)
            recycle = self.recycle_output and g.numel() > ops.TOPK_SMALL_N
            out, prev_idx = self._recycler.take(name, g) if recycle else (None, None)
            _, _, idx, out = ops.topk_step_dense(g, ops.ratio_k(g.numel(), self.compress_ratio), out=out,
                                                 prev_idx=prev_idx)
            if recycle:
                self._recycler.keep(name, out, idx)
            return out.view(tensor.shape)
        if not (isinstance(communicator, Allgather) and type(mem) is ResidualMemory
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        g = ops.dev_f32(tensor)
        n = g.numel()
        k = ops.ratio_k(n, self.compress_ratio)
        res = mem.residuals.get(name)
        has = res is not None and res.numel() == n and res.device == g.device
        if not has:
            res = torch.empty_like(g)
        world = int(communicator.world_size)
        carry, carry_valid = mem.carry_for(name, res, has, k)
        if world == 1:
            recycle = self.recycle_output == "always" and n > ops.TOPK_SMALL_N
            # a large bucket's first step takes the residual and output allocations that stream fastest
            # together (ops.pick_pair: the pair of allocations decides the main pass's rate); the name
            # keeps that output buffer (its dropped previous result comes back, rewritten densely)
            place = (not recycle and self.recycle_output is not False and ops.PLACE_PROBE
                     and n >= ops.PLACE_MIN_N)
            if recycle:
                out, prev_idx = self._recycler.take(name, g)
            elif place:
                out, _ = self._recycler.take(name, g, dense=True)
                prev_idx = None   # dense rewrite: every element of out is written
            else:
                out, prev_idx = torch.empty_like(g), None
            if place and not has:
                res, out, probes = ops.pick_pair(g)
                if probes:
                    self.place_probes[name] = probes
                carry, carry_valid = mem.carry_for(name, res, has, k)
            _, _, idx = ops.topk_residual_step(g, res, has, mem.beta, mem.gamma, k, out=out, carry=carry,
                                               carry_valid=carry_valid, prev_idx=prev_idx)
            mem.residuals[name] = res
            mem.carry_written(name, res, carry)
            if recycle or place:
                self._recycler.keep(name, out, idx)
            return out.view(tensor.shape)   # (0 + d) / 1: the fused kernel writes exactly this
        # world > 1: the new residual goes to a second buffer (no dense output to park t in), so the
        # main pass zeroes its provisional picks at once (grace_topk_residual_step_swap)
        if getattr(mem, "keep_spare", True):
            res_new = mem.spare_for(name, g)
            buf, vals, idx = ops.topk_residual_step_swap(g, res if has else None, has, mem.beta, mem.gamma, k,
                                                         res_new, carry=carry, carry_valid=carry_valid)
            mem.retire(name, res if has else None)
            mem.residuals[name] = res_new
            mem.carry_written(name, res_new, carry)
        else:
            # ResidualMemory(keep_spare=False): one residual buffer per name, updated in place (4 B
            # per parameter less; the finalize zeroes the selected positions instead)
            buf, vals, idx = ops.topk_residual_step(g, res, has, mem.beta, mem.gamma, k, out=None, carry=carry,
                                                    carry_valid=carry_valid)
            mem.residuals[name] = res
            mem.carry_written(name, res, carry)
        divisor = world if self.average else 1
        if n > ops.SORT_PAYLOAD_MAX_N:
            # beyond the index-sorted grouping's range (payload.hip): gather as-is and decode with
            # the rank-ordered scatter-accumulate instead
            gathered = torch.empty(world * 2 * k, dtype=torch.float32, device=g.device)
            dist.all_gather_into_tensor(gathered, buf)
            out = ops.sparse_aggregate(gathered, gathered[k:].view(torch.int32), 2 * k, [k] * world, world, n,
                                       divisor)
            return out.view(tensor.shape)
        # sort the local payload by index, exchange, then decode all W payloads in one pass over the
        # output (grace_amd/csrc/payload.hip) instead of W random scatters
        sbuf = ops.sort_payload(buf, k, n)
        gathered = torch.empty(world * sbuf.numel(), dtype=torch.float32, device=g.device)
        dist.all_gather_into_tensor(gathered, sbuf)
        out = ops.sparse_aggregate_sorted(gathered, k, world, n, divisor)
        return out.view(tensor.shape)
