"""Per-tensor top-k + residual for a whole model in one launch sequence.

The reference's DDP loop (examples/dist/CIFAR10-dawndist/core.py:203-206) calls
``Allgather(TopKCompressor(ratio), ResidualMemory(), W).step(grad, name)`` once per parameter: every
tensor gets its own k_i = max(1, int(n_i * ratio)) (grace_dl/dist/compressor/topk.py:34) and its
own residual (grace_dl/dist/memory/residual.py:10-20).  ``SegmentedTopK.step`` computes exactly
that for all tensors at once -- they are segments of one flat gradient buffer (harness.GradBucket)
-- with three launches that stream every element once (grace_amd/csrc/topk.hip "Segmented": small
tensors selected exactly in one workgroup each, large ones through the single-bucket engine's
sampled bracket, main pass and finalize, per segment) instead of three launches per tensor.  At W > 1 the
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
        self._sizes_memo = None   # (snapshot of the last `sizes`, its total, its int tuple)
        self.last_payload = None
        # A/B knobs (tools/ab_seg.py): the small-segment limit (<= the library's kSmallN) and the
        # order of the large segments' chunks ("index": tensor order; "size": descending size, which
        # measured 0.4-4 us slower per step on the ResNet-50 set)
        self._small_max = None
        self._order = "index"
        # per name: the residual-sample carry of the large segments (the bracket reads g alone at
        # its sample positions when the carry holds the previous step of the same residual), the
        # residual and its version counter when the carry was written, the tables it belongs to
        self._carries = {}
        self._use_carry = True   # A/B knob (tools/ab_seg.py)

    def tables(self, sizes, device, has_res, dense_out):
        """Device tables of one segment list (cached): offsets, the small / large split, the main
        pass's chunk map of the large segments (its chunk length follows the bytes per element, so
        it depends on has_res and on the dense output) and their workspaces.  Per stream as well:
        the workspaces' counters are re-zeroed by the next launch on the same stream, so two streams
        must never share one."""
        memo = self._sizes_memo
        if memo is None or sizes is not memo[2]:   # local_step passes the memoised tuple itself
            sizes = tuple(int(n) for n in sizes)
        key = (sizes, str(device), ops._stream(), bool(has_res), bool(dense_out))
        hit = self._tables.get(key)
        if hit is not None:
            return hit
        small_max = int(self._small_max or _lib.query("grace_topk_segmented_small_max"))
        chunk = int(_lib.query("grace_topk_segmented_chunk", 1 if has_res else 0, 1 if dense_out else 0))
        seg, kk = [0], [0]
        large, small, chk, chunk_li, ws_off, fin, fin_li = [], [], [0], [], [], [0], []
        ws_total = 0
        carry_off, carry_total = [], 0
        ks = []
        for i, n in enumerate(sizes):
            if n < 1:
                raise ValueError("empty tensor in the segment table")
            k = min(n, ops.ratio_k(n, self.compress_ratio))        # torch.topk needs k <= n
            ks.append(k)
            seg.append(seg[-1] + n)
            kk.append(kk[-1] + k)
            if n <= small_max:
                small.append(i)
        order = (lambda i: (-sizes[i], i)) if self._order == "size" else (lambda i: i)
        for i in sorted((i for i, n in enumerate(sizes) if n > small_max), key=order):
            n, k = sizes[i], ks[i]
            li = len(large)
            large.append(i)
            c = (n + chunk - 1) // chunk
            chk.append(chk[-1] + c)
            chunk_li += [li] * c
            ws_off.append(ws_total)
            f = int(_lib.query("grace_topk_segmented_fin_blocks", n, k))
            fin.append(fin[-1] + f)
            fin_li += [li] * f
            ws_total += (int(_lib.query("grace_topk_segmented_seg_ws_bytes", n, k)) + 255) // 256 * 256
            carry_off.append(carry_total)
            carry_total += (int(_lib.query("grace_topk_segmented_carry_len", n)) + 3) // 4 * 4   # 16-B aligned
        import ctypes
        ln = (ctypes.c_int64 * max(1, len(large)))(*[sizes[i] for i in large])
        lk = (ctypes.c_int64 * max(1, len(large)))(*[ks[i] for i in large])
        ws_need = int(_lib.query("grace_topk_segmented_workspace_bytes", ctypes.addressof(ln), ctypes.addressof(lk),
                                 len(large)))
        if ws_need != ws_total:
            raise RuntimeError(f"segmented workspace layout mismatch: {ws_need} != {ws_total}")
        t64 = lambda v: torch.tensor(v, dtype=torch.int64).to(device)   # noqa: E731
        t32 = lambda v: torch.tensor(v, dtype=torch.int32).to(device)   # noqa: E731
        ws = torch.zeros(max(ws_total, 256), dtype=torch.uint8, device=device)
        hit = {"seg_off": t64(seg), "k_off": t64(kk), "large": t32(large or [0]), "n_large": len(large),
               "small": t32(small or [0]), "n_small": len(small), "chk_off": t64(chk), "chunk_li": t32(chunk_li or [0]),
               "nchunks": chk[-1], "ws_off": t64(ws_off or [0]), "fin_off": t64(fin), "fin_li": t32(fin_li or [0]),
               "nfin": fin[-1], "ws": ws, "k_total": kk[-1], "n": seg[-1],
               "carry_off": t64(carry_off or [0]), "carry_len": max(carry_total, 4),
               "carry_key": (sizes, small_max),   # the carry layout depends on these only
               "ws_need": ws_need}
        hit["args"] = (hit["seg_off"].data_ptr(), hit["k_off"].data_ptr(), hit["large"].data_ptr(), hit["n_large"],
                       hit["small"].data_ptr(), hit["n_small"], hit["chk_off"].data_ptr(), hit["chunk_li"].data_ptr(),
                       hit["nchunks"], hit["ws_off"].data_ptr(), hit["fin_off"].data_ptr(), hit["fin_li"].data_ptr(),
                       hit["nfin"], hit["n"])
        self._tables[key] = hit
        return hit

    def local_step(self, flat, sizes, name="bucket", dense=None):
        """This rank's half of the step: every tensor's compensate + top-k + residual update, the
        payload (vals, GLOBAL idx) in self.last_payload, and the dense result into `dense` when
        given (world 1; may be ``flat`` itself).  Returns the packed payload [vals | idx]."""
        g = ops.dev_f32(flat)
        n = g.numel()
        total, sizes = self._norm_sizes(sizes)
        if total != n:
            raise ValueError("segment sizes do not add up to the buffer")
        res = self.residuals.get(name)
        has = res is not None and res.numel() == n
        if not has:
            res = torch.empty_like(g)
            self.residuals[name] = res
        T = self.tables(sizes, g.device, has, dense is not None)
        k_total = T["k_total"]
        pay = torch.empty(2 * k_total, dtype=torch.float32, device=g.device)
        vals, idx = pay[:k_total], pay[k_total:].view(torch.int32)
        carry, valid = self._carry_for(name, res, has, T) if self._use_carry else (None, False)
        _lib.call("grace_topk_segmented_step", g.data_ptr(), res.data_ptr(), 1 if has else 0, self.beta, self.gamma,
                  *T["args"], vals.data_ptr(), idx.data_ptr(),
                  dense.data_ptr() if dense is not None else None,
                  carry.data_ptr() if carry is not None else None, T["carry_off"].data_ptr(), 1 if valid else 0,
                  T["ws"].data_ptr(), T["ws"].numel(), T["ws_need"], ops._stream())
        if carry is not None:   # written by this step (the kernels only use it with a residual)
            self._carries[name] = (carry, res, res._version, T["carry_key"])
        self.last_payload = (vals, idx)
        return pay

    def _norm_sizes(self, sizes):
        """(total, tuple of ints) of a segment list.  A step is launch-bound on the host side
        (~100 us of Python per step against ~90 us of device time on the ResNet-50 set), so the
        161-element conversion is memoised: a list or tuple equal to the previous call's (one
        C-level compare) reuses its result."""
        memo = self._sizes_memo
        if memo is not None and type(sizes) is type(memo[0]) and sizes == memo[0]:
            return memo[1], memo[2]
        t = tuple(int(n) for n in sizes)
        snap = list(sizes) if isinstance(sizes, list) else (tuple(sizes) if isinstance(sizes, tuple) else None)
        total = sum(t)
        if snap is not None:
            self._sizes_memo = (snap, total, t)
        return total, t

    def _carry_for(self, name, res, has, T):
        """This name's carry buffer and whether it holds the previous step of `res` as that step
        left it: the same residual tensor, unmodified since (version counter), the same segment
        layout (sizes and small-segment limit; the tables also differ by has_res, the carry not)."""
        ent = self._carries.get(name)
        if ent is not None and ent[0].numel() == T["carry_len"] and ent[0].device == res.device:
            carry = ent[0]
            valid = bool(has) and ent[1] is res and ent[2] == res._version and ent[3] == T["carry_key"]
        else:
            carry = torch.empty(T["carry_len"], dtype=torch.float32, device=res.device)
            valid = False
        return carry, valid

    def step(self, flat, sizes, name="bucket", out=None):
        """flat: f32[sum(sizes)] gradients; returns the flat aggregated result (``out`` if given,
        which may be ``flat`` itself: every tensor's result lands in place)."""
        W = int(self.world_size)
        if W == 1:
            dense = out if out is not None else torch.empty_like(ops.dev_f32(flat))
            self.local_step(flat, sizes, name, dense)
            return dense
        pay = self.local_step(flat, sizes, name, None)
        k_total = pay.numel() // 2
        n = flat.numel()
        gathered = torch.empty(W * 2 * k_total, dtype=torch.float32, device=pay.device)
        dist.all_gather_into_tensor(gathered, pay)
        return ops.sparse_aggregate(gathered, gathered[k_total:].view(torch.int32), 2 * k_total, [k_total] * W, W, n,
                                    W if self.average else 1, out=None if out is None else ops.fill(out, 0.0))
