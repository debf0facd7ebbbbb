"""Sharded top-k with residual error feedback: ONE gradient bucket split into contiguous shards,
one per rank (BASELINE configs[4]: 256 MiB bucket, k = 0.1 %, 8 x MI355X).

The reference has no sharded mode -- its Allgather (grace_dl/dist/communicator/allgather.py:8-45)
runs every rank on its own full bucket.  Here each rank owns n/W elements and the ranks together
select exactly the single-GPU top-k of the whole bucket (TopKCompressor, topk.py:32-42, with the
same tie rule as the single-GPU engine: larger |t| first, lower global index first), keep the
residual of their own shard (ResidualMemory, residual.py:10-20) and decode the replicated dense
bucket (or only their own slice, ``dense="shard"``).

Per step (kernels: grace_amd/csrc/topk.hip, "Sharded top-k"):
  1. sample this shard's |t| into the shared bracket histogram xs      -> all_reduce(xs)
  2. global bracket + one streaming pass over the shard (t, r' = t, local candidates)
                                                                       -> all_gather(xh)
  3. host: boundary bin B, how many of it are still needed, exact list capacities (one 8 KB/rank
     read -- the step's only host synchronisation)
  4. route: sure + above-B entries to the local payload, bin-B entries to a list
                                                                       -> all_gather(lists)
  5. boundary: exact global ranking of bin B; winners join their owner's payload
                                                                       -> all_gather(payloads)
  6. scatter-range decode into the dense output.
If the sampled bracket misses (degenerate data: heavy ties, mostly-zero buckets) every rank
gathers t and runs the exact single-GPU selection instead (same result, slower).

``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator of the
same six calls to run the protocol on gloo.
"""
import numpy as np
import torch
import torch.distributed as dist

from grace_amd import ops

HIST_BINS = 2048


class NativeShardKernels:
    """The HIP kernels behind each protocol step (GPU tensors only)."""

    def exchange_buffers(self, device):
        return ops.shard_exchange_buffers(device)

    def empty(self, n, dtype, device):
        return torch.empty(n, dtype=dtype, device=device)

    def cand_cap(self, m, k):
        return min(m, 2 * k + 65536)   # topk.hip topk_cap

    sample = staticmethod(ops.shard_sample)
    main = staticmethod(ops.shard_main)
    route = staticmethod(ops.shard_route)
    boundary = staticmethod(ops.shard_boundary)
    take = staticmethod(ops.shard_take)
    scatter_range = staticmethod(ops.scatter_range)

    def fill_zero(self, x):
        return ops.fill(x, 0.0)

    def select_all(self, t, k):
        _, vals, idx = ops.topk_compress(t, k)
        return vals, idx


def plan_boundary(xh_all, k, world, cand_cap):
    """Host step 3 from the gathered [W, 2048 + 8] exchange rows (hist, n_sure, n_cand, ...).

    Returns (ok, B, need, cap_b, cap_p): B the boundary bin (2048 when no candidate is needed),
    need the count still to take from bin B, cap_b the largest per-rank bin-B list, cap_p an upper
    bound of any rank's payload count.  ok False = the bracket missed or a list overflowed."""
    xh_all = np.asarray(xh_all, dtype=np.int64).reshape(world, -1)
    hist_r = xh_all[:, :HIST_BINS]
    n_sure_r = xh_all[:, HIST_BINS]
    n_cand_r = xh_all[:, HIST_BINS + 1]
    s = int(n_sure_r.sum())
    c = int(n_cand_r.sum())
    if s > k or s + c < k or bool((n_cand_r > cand_cap).any()):
        return False, -1, 0, 0, 0
    target = k - s
    if target == 0:
        return True, HIST_BINS, 0, 0, int(n_sure_r.max())
    hist = hist_r.sum(axis=0)
    above_incl = np.cumsum(hist[::-1])[::-1]          # count in bins >= b
    above = above_incl - hist                          # count in bins > b
    cand = np.nonzero((above < target) & (target <= above_incl))[0]
    B = int(cand.max())
    need = int(target - above[B])
    cap_b = int(hist_r[:, B].max())
    cap_p = int(min(k, (n_sure_r + (hist_r[:, B:].sum(axis=1))).max()))
    return True, B, need, cap_b, cap_p


class ShardedTopK:
    """Top-k (ratio) + residual memory over one bucket sharded across the ranks of `group`."""

    def __init__(self, compress_ratio, group=None, dense="replicated", kernels=None):
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        self.compress_ratio = compress_ratio
        self.group = group
        self.dense = dense
        self.k_ops = kernels or NativeShardKernels()
        self.residuals = {}
        self._sizes = {}
        self.last_payload = None      # (vals, idx) of this rank's entries of the last step
        self.last_fallback = False
        self.resizes = 0              # steps that found a rank's shard resized (and were redone)

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def _shard_sizes(self, name, m, device, world):
        """Shard sizes of `name` on every rank.  Exchanged on a name's first step only; every later
        step re-checks them for free through the shard length each rank's main pass writes into
        its exchanged counters (step 3), so a resize on any rank is seen by ALL ranks in the same
        step and they take the same branch (no rank-local collective)."""
        sizes = self._sizes.get(name)
        if sizes is None:
            if world > 1:
                mine = torch.tensor([m], dtype=torch.int64, device=device)
                allm = self.k_ops.empty(world, torch.int64, device)
                dist.all_gather_into_tensor(allm, mine, group=self.group)
                sizes = [int(v) for v in allm.cpu().tolist()]
            else:
                sizes = [m]
            self._sizes[name] = sizes
        return sizes

    def step(self, shard, name):
        return self._step(shard.reshape(-1), name, compensated=False)

    def _step(self, g, name, compensated):
        """compensated=True: g already is t = beta r + gamma g (the redo after a resize)."""
        K = self.k_ops
        world, rank = self._world()
        dev = g.device
        m = g.numel()
        sizes = self._shard_sizes(name, m, dev, world)
        base = sum(sizes[:rank])
        n = sum(sizes)
        k = ops.ratio_k(n, self.compress_ratio)
        res = self.residuals.get(name)
        has_res = res is not None and res.numel() == m and not compensated
        if res is None or res.numel() != m:
            res = K.empty(m, torch.float32, dev)
        self.residuals[name] = res
        stratum = max(1, n // ops.SAMPLE_MAX)
        sample_total = sum(sz // stratum for sz in sizes)
        xs, xh = K.exchange_buffers(dev)
        vals = K.empty(k, torch.float32, dev)
        idx = K.empty(k, torch.int32, dev)

        K.sample(g, res, has_res, stratum, xs)
        if world > 1:
            dist.all_reduce(xs, group=self.group)
        K.main(g, res, has_res, base, n, k, sample_total, vals, idx, xs, xh)
        if world > 1:
            xh_all = K.empty(world * xh.numel(), torch.int32, dev)
            dist.all_gather_into_tensor(xh_all, xh, group=self.group)
        else:
            xh_all = xh
        # the exchange rows go to the host asynchronously; the dense output's zero-fill is queued
        # behind them, so it runs on the GPU while the host plans the boundary
        host = self._host_rows(xh_all)
        out_len = m if self.dense == "shard" else n
        out = K.fill_zero(K.empty(out_len, torch.float32, dev))
        self._wait_host()
        rows = host.numpy().reshape(world, -1)
        seen = [int(v) for v in rows[:, HIST_BINS + 2]]
        if seen != list(sizes):
            # some rank's shard changed size: this pass ran on stale offsets.  Every rank sees the
            # same gathered lengths, so all of them redo the step with the new sizes.  The main
            # pass left t = beta r + gamma g in the residual buffer, so the redo starts from a copy
            # of t as an already-compensated gradient: a rank whose shard kept its size keeps its
            # error feedback exactly (residual.py:10-14 applied once), a resized rank starts from
            # t = g as on a first step.  Counted in ``resizes``.
            self._sizes[name] = seen
            self.resizes += 1
            return self._step(res.clone(), name, compensated=True)
        ok, B, need, cap_b, cap_p = plan_boundary(rows, k, world, K.cand_cap(m, k))
        self.last_fallback = not ok
        if not ok:
            return self._fallback(res, base, n, k, sizes, world, vals, idx, dev, out)

        bsend = K.empty(cap_b + 1, torch.int64, dev)
        K.route(res, base, k, B, vals, idx, bsend)
        if world > 1:
            brecv = K.empty(world * (cap_b + 1), torch.int64, dev)
            dist.all_gather_into_tensor(brecv, bsend, group=self.group)
        else:
            brecv = bsend
        K.boundary(res, base, k, brecv, world, cap_b, need, vals, idx, cap_p)
        self.last_payload = (vals[:cap_p], idx[:cap_p])
        return self._decode(vals, idx, cap_p, base, n, m, world, dev, out)

    def _host_rows(self, xh_all):
        """Start the device->host copy of the exchange rows (pinned, non-blocking)."""
        if not xh_all.is_cuda:
            self._evt = None
            return xh_all
        buf = getattr(self, "_pinned", None)
        if buf is None or buf.numel() != xh_all.numel():
            buf = torch.empty(xh_all.numel(), dtype=xh_all.dtype, pin_memory=True)
            self._pinned = buf
        buf.copy_(xh_all, non_blocking=True)
        self._evt = torch.cuda.Event()
        self._evt.record()
        return buf

    def _wait_host(self):
        if self._evt is not None:
            self._evt.synchronize()

    def _decode(self, vals, idx, cap_p, base, n, m, world, dev, out):
        K = self.k_ops
        if self.dense == "shard":
            K.scatter_range(vals, idx, 0, cap_p, 1, base, out)
            return out
        if world == 1:
            K.scatter_range(vals, idx, 0, cap_p, 1, 0, out)
            return out
        send = K.empty(2 * cap_p, torch.float32, dev)
        send[:cap_p].copy_(vals[:cap_p])
        send[cap_p:].copy_(idx[:cap_p].view(torch.float32))
        recv = K.empty(world * 2 * cap_p, torch.float32, dev)
        dist.all_gather_into_tensor(recv, send, group=self.group)
        K.scatter_range(recv, recv[cap_p:].view(torch.int32), 2 * cap_p, cap_p, world, 0, out)
        return out

    def _fallback(self, res, base, n, k, sizes, world, vals, idx, dev, out):
        """Exact path: the residual buffer holds t for every element after the main pass."""
        K = self.k_ops
        if world > 1:
            if len(set(sizes)) != 1:
                # unequal shards: RCCL / gloo gathers need one size, so pad every shard to the
                # largest and cut the padding out of the gathered rows
                mx = max(sizes)
                send = K.empty(mx, torch.float32, dev)
                send[:res.numel()].copy_(res)
                recv = K.empty(world * mx, torch.float32, dev)
                dist.all_gather_into_tensor(recv, send, group=self.group)
                t_all = torch.cat([recv[r * mx:r * mx + sz] for r, sz in enumerate(sizes)])
            else:
                t_all = K.empty(n, torch.float32, dev)
                dist.all_gather_into_tensor(t_all, res, group=self.group)
        else:
            t_all = res.clone()
        vals_all, idx_all = K.select_all(t_all, k)
        K.take(vals_all, idx_all, k, res, base, vals, idx, k)
        self.last_payload = (vals, idx)
        K.scatter_range(vals_all, idx_all, 0, k, 1, base if self.dense == "shard" else 0, out)
        return out
