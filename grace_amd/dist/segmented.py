"""Per-tensor top-k + residual for a whole model in one launch sequence.

The reference's DDP loop (examples/dist/CIFAR10-dawndist/core.py:203-206) calls
``Allgather(TopKCompressor(ratio), ResidualMemory(), W).step(grad, name)`` once per parameter: every
tensor gets its own k_i = max(1, int(n_i * ratio)) (grace_dl/dist/compressor/topk.py:34) and its
own residual (grace_dl/dist/memory/residual.py:10-20).  ``SegmentedTopK.step`` computes exactly
that for all tensors at once -- they are segments of one flat gradient buffer (harness.GradBucket)
-- with four launches (grace_amd/csrc/segtopk.hip) instead of three per tensor.  At W > 1 the
concatenated payloads (global indices) move in ONE all-gather and are decoded + aggregated in rank
order into the flat output (allgather.py:40-45 per tensor = per element of the flat buffer).

This is NOT the one-bucket variant (harness.step_bucketed), which runs one global top-k over the
concatenation -- a different algorithm.
"""
import torch
import torch.distributed as dist

from grace_amd import _lib, ops


class SegmentedTopK:

    def __init__(self, compress_ratio, world_size=1, average=True):
        self.compress_ratio = compress_ratio
        self.world_size = world_size
        self.average = average
        self.beta, self.gamma = 1.0, 1.0
        self.residuals = {}
        self._tables = {}
        self.last_payload = None

    def tables(self, sizes, device):
        # per stream as well: the workspace's histograms and counters are re-zeroed by the next
        # launch on the same stream, so two streams must never share one
        key = (tuple(int(s) for s in sizes), str(device), ops._stream())
        hit = self._tables.get(key)
        if hit is None:
            chunk = _lib.query("grace_topk_segmented_chunk")
            seg, kk, chk, cseg = [0], [0], [0], []
            for i, n in enumerate(key[0]):
                if n < 1:
                    raise ValueError("empty tensor in the segment table")
                seg.append(seg[-1] + n)
                kk.append(kk[-1] + min(n, ops.ratio_k(n, self.compress_ratio)))   # torch.topk needs k <= n
                c = (n + chunk - 1) // chunk
                chk.append(chk[-1] + c)
                cseg += [i] * c
            t64 = lambda v: torch.tensor(v, dtype=torch.int64).to(device)   # noqa: E731
            ws = torch.zeros(_lib.query("grace_topk_segmented_workspace_bytes", seg[-1], len(key[0])),
                             dtype=torch.uint8, device=device)
            hit = (t64(seg), t64(kk), t64(chk), torch.tensor(cseg, dtype=torch.int32).to(device), kk[-1], chk[-1], ws)
            self._tables[key] = hit
        return hit

    def step(self, flat, sizes, name="bucket", out=None):
        """flat: f32[sum(sizes)] gradients; returns the flat aggregated result (``out`` if given,
        which may be ``flat`` itself: every tensor's result lands in place)."""
        g = ops.dev_f32(flat)
        n = g.numel()
        seg_off, k_off, chk_off, chunk_seg, k_total, nchunks, ws = self.tables(sizes, g.device)
        if sum(int(s) for s in sizes) != n:
            raise ValueError("segment sizes do not add up to the buffer")
        res = self.residuals.get(name)
        has = res is not None and res.numel() == n
        if not has:
            res = torch.empty_like(g)
            self.residuals[name] = res
        pay = torch.empty(2 * k_total, dtype=torch.float32, device=g.device)
        vals, idx = pay[:k_total], pay[k_total:].view(torch.int32)
        W = int(self.world_size)
        dense = (out if out is not None else torch.empty_like(g)) if W == 1 else None
        _lib.call("grace_topk_segmented_step", g.data_ptr(), res.data_ptr(), 1 if has else 0, self.beta, self.gamma,
                  seg_off.data_ptr(), k_off.data_ptr(), chk_off.data_ptr(), chunk_seg.data_ptr(), len(sizes), n,
                  nchunks, vals.data_ptr(), idx.data_ptr(), dense.data_ptr() if dense is not None else None,
                  ws.data_ptr(), ws.numel(), ops._stream())
        self.last_payload = (vals, idx)
        if W == 1:
            return dense
        gathered = torch.empty(W * 2 * k_total, dtype=torch.float32, device=g.device)
        dist.all_gather_into_tensor(gathered, pay)
        return ops.sparse_aggregate(gathered, gathered[k_total:].view(torch.int32), 2 * k_total, [k_total] * W, W, n,
                                    W if self.average else 1, out=None if out is None else ops.fill(out, 0.0))
