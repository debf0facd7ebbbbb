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

Variable-size exchange at world size W > 1 (``fused_step``, Allgather + DgcMemory).  The reference
syncs the host twice per step: ``torch.where`` sizes the payload (dgc.py:37-40) and Allgather reads
the gathered sizes back (allgather.py:15-18).  Here the count never leaves the device before the
exchange, as for ThresholdCompressor:
  * ``exchange="counts"`` (default): the W device counts are all-gathered and read ONCE, then one
    fixed-size record per rank (capacity = the largest count) moves in one all-gather;
  * ``exchange="capacity"``: the record capacity is the name's previous largest count x
    ``capacity_margin``, so the common step reads nothing on the host.  On overflow (a rank selected
    more than the capacity) ``overflow="retry"`` (default) reads the stat once at the end of the step
    and redoes an overflowing step through the counts exchange (bit-exact always, like Threshold);
    ``overflow="defer"`` sends the first ``cap`` entries in index
    order and leaves the rest in the momentum memory -- DgcMemory.update zeroes r and a only where an
    entry travelled, so the unsent ones are selected again later (error feedback); the overflow stat
    is copied asynchronously and grows the capacity at the name's next step (a departure from the
    reference step, so it is opt-in and warns once when it first defers).
Without overflow every mode equals the reference's four calls bit for bit (the decode is the
rank-ordered scatter-add of sparse.hip, divided once per element).
"""
import warnings

import numpy as np
import torch
import torch.distributed as dist

from grace_amd import ops
from grace_amd.dist import Compressor


class DgcCompressor(Compressor):
    _warned_defer = False

    def __init__(self, compress_ratio, rng="device", exchange="counts", capacity_margin=1.25, overflow="retry"):
        super().__init__(tensors_size_are_same=False)
        if exchange not in ("counts", "capacity") or overflow not in ("retry", "defer"):
            raise ValueError("exchange must be 'counts' or 'capacity', overflow 'retry' or 'defer'")
        if not capacity_margin >= 1.0:
            raise ValueError("capacity_margin must be >= 1")
        self.compress_ratio = compress_ratio
        self.rng = rng
        self.exchange = exchange
        self.capacity_margin = float(capacity_margin)
        self.overflow = overflow
        self.capacity = {}        # name -> record capacity (entries per rank)
        self._pending = {}        # name -> (pinned stat, event) of a deferred step
        self.overflows = 0        # capacity overflows seen (deferred or retried)
        self.host_reads = 0       # blocking host reads issued by fused_step (diagnostic)
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
        if not (type(communicator) is Allgather and type(mem) is DgcMemory
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        W = int(communicator.world_size)
        if W == 1 and not mem.gradient_clipping:
            # one streaming pass from the old state into new buffers (the reference rebinds new
            # tensors too, memory/dgc.py:36-39): compensate + select + mask + (0 + decompress) / 1
            g = ops.dev_f32(tensor)
            res, acc = mem.residuals.get(name), mem.gradients.get(name)
            has = res is not None and acc is not None and res.numel() == g.numel() and acc.numel() == g.numel()
            sidx, seed = self._sampling(g, name)
            out, r_new, a_new = ops.dgc_step_w1_fused(g, res if has else None, acc if has else None, has,
                                                      mem.momentum, self.compress_ratio, sample_idx=sidx, seed=seed)
            mem.residuals[name], mem.gradients[name] = r_new, a_new
            return out.view(tensor.shape)
        if W > 1 and tensor.numel() >= 2 ** 31:
            return None        # grace_dgc_write_capped indexes with int32: the generic path handles it
        t = ops.dev_f32(mem.compensate(tensor, name))
        sidx, seed = self._sampling(t, name)
        if W == 1:
            ws = ops.dgc_select(t, self.compress_ratio, sample_idx=sidx, seed=seed)
            out = ops.dgc_step_w1(t, mem.residuals[name], mem.gradients[name], ws)
            return out.view(tensor.shape)
        return self._exchange_step(t, name, mem, W, sidx, seed).view(tensor.shape)

    # ------------------------------------------------------------------ world size > 1
    def _grow(self, max_count, n):
        return int(min(n, max(64, int(np.ceil(max_count * self.capacity_margin)))))

    def _settle(self, name, n):
        """Deferred mode: the previous step's stat (long finished) resizes the capacity."""
        pend = self._pending.pop(name, None)
        if pend is None:
            return
        pinned, ev = pend
        ev.synchronize()
        mx, over = (int(v) for v in pinned.tolist())
        if over:
            self.overflows += 1
            if not DgcCompressor._warned_defer:
                DgcCompressor._warned_defer = True
                warnings.warn("grace_amd DgcCompressor(overflow='defer'): a step selected more entries than the "
                              "record capacity; the unsent ones stay in the momentum memory (not the reference "
                              "step; use overflow='retry' for bit-exact steps)", RuntimeWarning, stacklevel=3)
        cap = self.capacity.get(name)
        if cap is not None and (over or self._grow(mx, n) * 4 < cap):
            self.capacity[name] = self._grow(mx, n)

    def _records(self, t, ws, cap, W):
        """Write this rank's record and all-gather the W records (rank-major)."""
        rec = ops.dgc_write_capped(t, ws, cap)
        recs = torch.empty(W * rec.numel(), dtype=torch.int32, device=t.device)
        dist.all_gather_into_tensor(recs, rec)
        return rec, recs

    def _exchange_step(self, t, name, mem, W, sidx, seed):
        n = t.numel()
        dev = t.device
        divisor = W if self.average else 1
        ws = ops.dgc_threshold_dev(t, self.compress_ratio, sample_idx=sidx, seed=seed)
        res, acc = mem.residuals[name], mem.gradients[name]
        defer = self.exchange == "capacity" and self.overflow == "defer"
        if defer:
            self._settle(name, n)
        cap = self.capacity.get(name) if self.exchange == "capacity" else None
        stat = torch.empty(2, dtype=torch.int32, device=dev)
        if cap is not None and cap <= n:
            rec, recs = self._records(t, ws, cap, W)
            out = ops.sparse_aggregate_capped(recs, cap, W, n, divisor, stat)
            if defer:
                ops.dgc_mask_update_capped(rec, cap, res, acc)
                pinned = torch.empty(2, dtype=torch.int32, pin_memory=True)
                pinned.copy_(stat, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._pending[name] = (pinned, ev)
                return out
            self.host_reads += 1
            mx, over = (int(v) for v in stat.cpu().tolist())        # one read, after the exchange
            if not over:
                ops.dgc_mask_update_capped(rec, cap, res, acc)
                if self._grow(mx, n) * 4 < cap:
                    self.capacity[name] = self._grow(mx, n)
                return out
            self.overflows += 1                                      # retry: memory still untouched
        # counts exchange: the W device counts, ONE host read, then records sized to the largest
        cnt = ws[8:12].view(torch.int32)
        counts_dev = torch.empty(W, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(counts_dev, cnt)
        self.host_reads += 1
        mx = max(int(c) for c in counts_dev.cpu().tolist())
        cap_exact = max(mx, 1)
        rec, recs = self._records(t, ws, cap_exact, W)
        out = ops.sparse_aggregate_capped(recs, cap_exact, W, n, divisor, stat)
        ops.dgc_mask_update_capped(rec, cap_exact, res, acc)
        if self.exchange == "capacity":
            self.capacity[name] = self._grow(mx, n)
        return out

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        shape, _, numel = ctx
        return ops.sparse_decode(values, indices, numel).view(shape)
