"""Threshold sparsification (grace_dl/dist/compressor/threshold.py:6-27): every element with
|x| >= min(threshold, max(x)) (signed max, as the reference), ascending index order, payload
[values f32[m], indices int32[m]] with m data-dependent (tensors_size_are_same=False).

Variable-size exchange.  The reference's step syncs the host twice: torch.where sizes the payload
(threshold.py:17) and Allgather exchanges the sizes as a CUDA tensor and reads them back
(allgather.py:15-18).  ``fused_step`` (Allgather with NoneMemory / ResidualMemory) offers:

* ``exchange="counts"`` (default): the count is finished on the device (recount decided there
  too), the W counts are all-gathered on the device, and ONE host read of those W counts sizes the
  local payload and the padded exchange buffer.
* ``exchange="capacity"``: a per-name capacity (the last max count x ``capacity_margin``) fixes the
  exchange size in advance; every rank all-gathers one fixed-size record {count, cap | vals | idx}
  and the aggregate reads the counts from the gathered headers on the device.  On overflow
  (some rank's count > cap) ``overflow="retry"`` redoes the step through the counts exchange after
  one read of the device stat at the END of the step (bit-exact always); ``overflow="defer"``
  (ResidualMemory only) reads nothing on the host: entries past the capacity are not sent and stay
  in the residual (error feedback), and the stat, copied asynchronously, grows the capacity at the
  name's next step.  Without overflow both are bit-exact with the reference."""
import numpy as np
import torch
import torch.distributed as dist

from grace_amd import _lib, ops
from grace_amd.dist import Compressor
from grace_amd.dist.communicator.allgather import Allgather
from grace_amd.dist.memory.none import NoneMemory
from grace_amd.dist.memory.residual import ResidualMemory


class ThresholdCompressor(Compressor):

    def __init__(self, threshold, exchange="counts", capacity_margin=1.25, overflow="retry"):
        super().__init__(tensors_size_are_same=False)
        if exchange not in ("counts", "capacity") or overflow not in ("retry", "defer"):
            raise ValueError("exchange must be 'counts' or 'capacity', overflow 'retry' or 'defer'")
        if not capacity_margin >= 1.0:
            raise ValueError("capacity_margin must be >= 1")
        self.threshold = threshold
        self.exchange = exchange
        self.capacity_margin = float(capacity_margin)
        self.overflow = overflow
        self.capacity = {}        # name -> exchange capacity (entries per rank)
        self._pending = {}        # name -> (pinned stat, event) of a deferred step
        self.overflows = 0        # capacity overflows seen (retried or deferred)
        # world-1 residual step on a large bucket: the residual / output allocation pair probed at
        # the first step and the output kept (rewritten in full), as TopKCompressor does (ops.pick_pair)
        self._recycler = ops.OutputRecycler()
        self.place_probes = {}

    def compress(self, tensor, name):
        values, indices = ops.threshold_compress(tensor, self.threshold)
        return [values, indices], tensor.size()

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        return ops.sparse_decode(values, indices, ctx.numel()).view(ctx)

    def decode_aggregate_variable(self, gathered, sizes, ctx, world_size):
        """Variable-size Allgather: rank-ordered scatter-add of the W padded payloads."""
        vals, idx = gathered
        if not vals.is_cuda:
            return None
        stride = vals.numel() // world_size
        counts = [int(sizes[r][0]) for r in range(world_size)]
        out = ops.sparse_aggregate(vals, idx, stride, counts, world_size, ctx.numel(),
                                   world_size if self.average else 1)
        return out.view(ctx)

    def _grow(self, max_count, n):
        return int(min(n, max(64, int(np.ceil(max_count * self.capacity_margin)))))

    def _counts_exchange(self, t, n, ws, W, dev):
        """One host read: the W device counts (allgather.py:15-18 without the per-tensor sync)."""
        cnt = ws[4:8].view(torch.int32)
        if W > 1:
            counts_dev = torch.empty(W, dtype=torch.int32, device=dev)
            dist.all_gather_into_tensor(counts_dev, cnt)
        else:
            counts_dev = cnt
        counts = [int(c) for c in counts_dev.cpu().tolist()]     # the step's ONE host read
        m, cap = counts[dist.get_rank() if W > 1 else 0], max(max(counts), 1)
        send = torch.empty(2 * cap, dtype=torch.float32, device=dev)     # [vals | idx], padded to the max
        vals, idx = send[:m], send[cap:cap + m].view(torch.int32)
        if m:
            _lib.call("grace_threshold_write", t.data_ptr(), n, ws.data_ptr(), vals.data_ptr(), idx.data_ptr(),
                      ops._stream())
        if W > 1:
            recv = torch.empty(W * 2 * cap, dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(recv, send)
            out = ops.sparse_aggregate(recv, recv[cap:].view(torch.int32), 2 * cap, counts, W, n,
                                       W if self.average else 1)
        else:
            out = ops.sparse_aggregate(send, send[cap:].view(torch.int32), 0, counts, 1, n, 1)
        return out, vals, idx, m, max(counts)

    def _settle(self, name, n):
        """Deferred mode: read the previous step's stat (long finished) and resize the capacity."""
        pend = self._pending.pop(name, None)
        if pend is None:
            return
        pinned, ev = pend
        ev.synchronize()
        mx, over = (int(v) for v in pinned.tolist())
        if over:
            self.overflows += 1
        cap = self.capacity.get(name)
        if cap is not None and (over or self._grow(mx, n) * 4 < cap):
            self.capacity[name] = self._grow(mx, n)

    def fused_step(self, communicator, tensor, name):
        mem = communicator.memory
        if not (communicator.__class__ is Allgather and type(mem) in (NoneMemory, ResidualMemory)
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        W = int(communicator.world_size)
        g = ops.dev_f32(tensor)
        n = g.numel()
        dev = g.device
        residual = type(mem) is ResidualMemory
        if W == 1 and self.exchange == "counts":
            # world 1: no payload at all -- t and the bound's statistics from one read, then one pass
            # for out = (0 + decompress) / 1 and r = t - decompress (grace_threshold_step_w1)
            ws = ops.workspace("threshold", _lib.query("grace_threshold_workspace_bytes", n), dev)
            place = residual and ops.PLACE_PROBE and n >= ops.PLACE_MIN_N
            out = self._recycler.take(name, g, dense=True)[0] if place else torch.empty_like(g)
            if residual:
                r = mem.residuals.get(name)
                has = r is not None and r.numel() == n and r.device == dev and r.is_contiguous()
                if not has and place:
                    buf, out, probes = ops.pick_pair(g)
                    if probes:
                        self.place_probes[name] = probes
                else:
                    buf = r.reshape(-1) if has else torch.empty_like(g)
                _lib.call("grace_threshold_step_w1", g.data_ptr(), buf.data_ptr(), 2 if has else 1, float(mem.beta),
                          float(mem.gamma), n, float(np.float32(self.threshold)), ws.data_ptr(), out.data_ptr(),
                          ops._stream())
                mem.residuals[name] = buf.view(tensor.shape)
                if place:
                    self._recycler.keep(name, out, None)
            else:
                _lib.call("grace_threshold_step_w1", g.data_ptr(), None, 0, 1.0, 1.0, n,
                          float(np.float32(self.threshold)), ws.data_ptr(), out.data_ptr(), ops._stream())
            return out.view(tensor.shape)
        # compensate (residual.py:10-14): t = beta r + gamma g, computed straight into the buffer that
        # becomes the new residual; the first step's t is the tensor itself (copied for the residual)
        if residual:
            r = mem.residuals.get(name)
            t = ops.axpby(r, g, mem.beta, mem.gamma) if r is not None and r.numel() == n else g.clone()
        else:
            t = g
        ws = ops.workspace("threshold", _lib.query("grace_threshold_workspace_bytes", n), dev)
        _lib.call("grace_threshold_count_dev", t.data_ptr(), n, float(np.float32(self.threshold)), ws.data_ptr(),
                  ops._stream())
        defer = self.overflow == "defer" and residual
        if defer:
            self._settle(name, n)
        cap = self.capacity.get(name) if self.exchange == "capacity" else None
        if cap is None or cap > n:
            out, vals, idx, m, mx = self._counts_exchange(t, n, ws, W, dev)
            if self.exchange == "capacity":
                self.capacity[name] = self._grow(mx, n)
            if residual:       # r = t - decompress(payload) (residual.py:16-20)
                _lib.call("grace_sparse_sub", vals.data_ptr(), idx.data_ptr(), m, t.data_ptr(), ops._stream())
                mem.residuals[name] = t.view(tensor.shape)
            return out.view(tensor.shape)
        # capacity-bounded: one fixed-size record per rank, no size round trip
        words = ops.exchange_record_words(cap)
        rec = torch.empty(words, dtype=torch.int32, device=dev)
        _lib.call("grace_threshold_write_capped", t.data_ptr(), n, ws.data_ptr(), rec.data_ptr(), cap, ops._stream())
        if W > 1:
            recs = torch.empty(W * words, dtype=torch.int32, device=dev)
            dist.all_gather_into_tensor(recs, rec)
        else:
            recs = rec
        stat = torch.empty(2, dtype=torch.int32, device=dev)
        out = ops.sparse_aggregate_capped(recs, cap, W, n, W if self.average else 1, stat)
        if defer:
            _lib.call("grace_sparse_sub_capped", rec.data_ptr(), cap, t.data_ptr(), ops._stream())
            mem.residuals[name] = t.view(tensor.shape)
            pinned = torch.empty(2, dtype=torch.int32, pin_memory=True)
            pinned.copy_(stat, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending[name] = (pinned, ev)
            return out.view(tensor.shape)
        mx, over = (int(v) for v in stat.cpu().tolist())        # one read, after the exchange
        if over:       # retry through the counts exchange; t (the residual-to-be) is still untouched
            self.overflows += 1
            out, vals, idx, m, mx = self._counts_exchange(t, n, ws, W, dev)
            self.capacity[name] = self._grow(mx, n)
            if residual:
                _lib.call("grace_sparse_sub", vals.data_ptr(), idx.data_ptr(), m, t.data_ptr(), ops._stream())
                mem.residuals[name] = t.view(tensor.shape)
            return out.view(tensor.shape)
        if self._grow(mx, n) * 4 < cap:
            self.capacity[name] = self._grow(mx, n)
        if residual:
            _lib.call("grace_sparse_sub_capped", rec.data_ptr(), cap, t.data_ptr(), ops._stream())
            mem.residuals[name] = t.view(tensor.shape)
        return out.view(tensor.shape)
