"""Sharded TernGrad: ONE bucket of tensors (a model's flat gradients with their segment table)
split over the ranks and compressed exactly as the single-GPU TernGradCompressor compresses every
tensor of it (grace_dl/dist/compressor/terngrad.py:7-30: per tensor its own 2.5 std clip and scalar,
codes in {-1, 0, 1}), then decoded.

A tensor's scale needs statistics of the whole tensor, which may span ranks.  The single-GPU codec
(csrc/quant.hip) already splits every tensor into 16384-element work units with f64 partials
(sum, sum of squares, max |x|, NaN) and reduces a tensor's unit partials in a fixed order.  So the
units are the partition, and the SURVEY's "one fp64 allreduce of (Σx, Σx², max|x|) per tensor"
becomes ONE all-gather of the unit partials: every rank then reduces the same partials in the same
order as the single-GPU encoder, and its scales are bit-identical to it, not just within ulps --
when every work unit starts on a multiple of 4 elements of the bucket (units of tensors whose
offsets are multiples of 4).  A unit at an odd offset is summed by the shard kernel in another quad
phase than by the whole-bucket kernel, so its f64 sum of squares may round differently: the clip
(2.5 std) and through it the scalar can then differ by an ulp, rarely.

Per step on rank r (grace_terngrad_shard_*, grace_terngrad_scalars):
  1. shard_stats: the partials of this rank's units into their slots of the global slot array;
  2. ONE all_gather_into_tensor of the slots (40 B per unit: 62 KB for ResNet-50's 1562 units);
  3. shard_encode: this rank's codes (the device generator keyed by GLOBAL element index, so the
     codes equal the single-GPU ones for the same seed, or an injected u); grace_terngrad_scalars:
     every tensor's scalar, derived on every rank -- nothing but the slots travels before the codes;
  4. dense="replicated": ONE all_gather of the codes and the decode of the whole bucket on every
     rank straight from the gathered per-rank records (grace_terngrad_decompress_records: no unpack
     pass, no copy into a flat code buffer); dense="shard": the decode of this rank's elements only,
     no second collective (reduce-scatter semantics).
Wire of step 4 (``wire``): "packed2" (default) moves the codes as code + 1 in the 2-bit planar byte
layout of the reference's packing (grace_dl/tensorflow/compressor/packing.py:4-29, grace_tern_pack /
grace_tern_unpack): a quarter of the int8 bytes over xGMI, unpacked straight into the flat code
buffer; "int8" moves the codes as they are (1 B per element).  The decoded result is the same.
Partition: the units in equal contiguous blocks (rank r: units [r U, (r + 1) U), U = ceil(units / W)),
so the slot all-gather lands every unit at its global index; partition() gives every rank's element
range and step() takes exactly that shard.  No host synchronisation in a step.

``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator.
"""
import torch
import torch.distributed as dist

from grace_amd import _lib, ops


class NativeTernKernels:
    """The HIP kernels behind each protocol step (GPU tensors only)."""

    def unit(self):
        return int(_lib.query("grace_terngrad_unit"))

    def new_slots(self, nslots, device):
        return torch.zeros((nslots, int(_lib.query("grace_terngrad_slot_bytes"))), dtype=torch.uint8, device=device)

    def tables(self, sizes, device):
        return ops.seg_tables(sizes, self.unit(), device)

    def stats(self, x, xoff, T, unit0, nu, slots):
        seg_off, unit_off, _ = T
        _lib.call("grace_terngrad_shard_stats", x.data_ptr(), int(xoff), seg_off.data_ptr(), unit_off.data_ptr(),
                  seg_off.numel() - 1, int(unit0), int(nu), slots.data_ptr(), ops._stream())

    def encode(self, x, xoff, T, unit0, nu, clip, u, seed, codes, slots):
        seg_off, unit_off, _ = T
        _lib.call("grace_terngrad_shard_encode", x.data_ptr(), int(xoff), seg_off.data_ptr(), unit_off.data_ptr(),
                  seg_off.numel() - 1, int(unit0), int(nu), ops._opt(clip), ops._opt(u), int(seed) & (2 ** 64 - 1),
                  codes.data_ptr(), slots.data_ptr(), ops._stream())

    def scalars(self, T, clip, slots, out):
        seg_off, unit_off, _ = T
        _lib.call("grace_terngrad_scalars", seg_off.data_ptr(), unit_off.data_ptr(), seg_off.numel() - 1,
                  ops._opt(clip), slots.data_ptr(), out.data_ptr(), ops._stream())

    def decode(self, codes, scalars, sizes, n):
        return ops.terngrad_decompress(codes, scalars, n, sizes)

    def seg_max(self):
        return int(_lib.query("grace_qsgd_seg_max"))

    def decode_records(self, records, rec_bytes, world, rank_lo, packed, scalars, sizes, n):
        """the whole bucket straight from the W gathered records, one launch (no unpack, no copy)"""
        return ops.terngrad_decompress_records(records, rec_bytes, world, rank_lo, packed, scalars, n, sizes)

    def pack_bytes(self, n):
        return int(_lib.query("grace_pack2_bytes", int(n)))

    def pack(self, codes, out):
        """codes (int8 {-1, 0, 1}) -> out[:pack_bytes(codes.numel())], the 2-bit layout of code + 1"""
        _lib.call("grace_tern_pack", codes.data_ptr(), codes.numel(), out.data_ptr(), ops._stream())

    def unpack(self, packed, n, out):
        """the first pack_bytes(n) bytes of packed -> n int8 codes into out"""
        _lib.call("grace_tern_unpack", packed.data_ptr(), int(n), out.data_ptr(), ops._stream())


class _Plan:
    """The unit partition of one segment table over `world` ranks."""

    def __init__(self, sizes, world, unit):
        self.sizes = tuple(int(s) for s in sizes)
        self.world = world
        starts = []                       # global element start of every unit
        seg = [0]
        for n in self.sizes:
            if n < 1:
                raise ValueError("ShardedTernGrad: empty tensor in the segment table")
            starts += [seg[-1] + j * unit for j in range((n + unit - 1) // unit)]
            seg.append(seg[-1] + n)
        self.n = seg[-1]
        self.seg = seg
        self.nunits = len(starts)
        starts.append(self.n)
        self.U = (self.nunits + world - 1) // world
        self.units = [(min(r * self.U, self.nunits), min((r + 1) * self.U, self.nunits)) for r in range(world)]
        self.ranges = [(starts[u0], starts[u1]) for u0, u1 in self.units]
        self.max_len = max(hi - lo for lo, hi in self.ranges)
        # per rank: the tensors its range touches (first, last) and their lengths inside it
        self.own = []
        for lo, hi in self.ranges:
            if hi == lo:
                self.own.append((0, 0, []))
                continue
            s0 = max(s for s in range(len(self.sizes)) if seg[s] <= lo)
            s1 = max(s for s in range(len(self.sizes)) if seg[s] < hi)
            self.own.append((s0, s1, [min(hi, seg[s + 1]) - max(lo, seg[s]) for s in range(s0, s1 + 1)]))


class ShardedTernGrad:
    """TernGrad over one bucket whose work units are sharded across the ranks of `group`."""

    def __init__(self, group=None, dense="replicated", kernels=None, seed=0, wire="packed2"):
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        if wire not in ("packed2", "int8"):
            raise ValueError("wire must be 'packed2' or 'int8'")
        self.group = group
        self.dense = dense
        self.wire = wire
        self.seed = seed
        self.k_ops = kernels or NativeTernKernels()
        self._plans = {}
        self._slots = {}
        self.last_codes = None      # this rank's codes (int8, its element range)
        self.last_scalars = None    # every tensor's scalar (f32[nseg]), identical on every rank

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def _plan(self, sizes, world):
        key = (tuple(int(s) for s in sizes), world)
        plan = self._plans.get(key)
        if plan is None:
            plan = self._plans[key] = _Plan(key[0], world, self.k_ops.unit())
        return plan

    def partition(self, sizes, world=None):
        """Every rank's [start, end) element range of the flat bucket (unit-aligned)."""
        return list(self._plan(sizes, world or self._world()[0]).ranges)

    def step(self, shard, sizes, clip=None, u=None, seed=None):
        """This rank's shard of the flat bucket (exactly partition(sizes)[rank], a 16-B aligned
        tensor of its own) -> the decoded bucket (dense="replicated") or this rank's decoded range
        (dense="shard").  clip: optional f32[nseg] injected clip bounds (global); u: optional f32
        uniform draws for THIS shard's elements."""
        K = self.k_ops
        world, rank = self._world()
        plan = self._plan(sizes, world)
        lo, hi = plan.ranges[rank]
        x = shard.reshape(-1)
        if x.numel() != hi - lo:
            raise ValueError(f"ShardedTernGrad: rank {rank} holds {x.numel()} elements, its unit range is {hi - lo} "
                             "(use partition(sizes))")
        dev = x.device
        T = K.tables(plan.sizes, dev)
        key = (plan.sizes, world, str(dev))
        slots = self._slots.get(key)
        if slots is None:
            slots = self._slots[key] = K.new_slots(world * plan.U + 1, dev)
        u0, u1 = plan.units[rank]
        K.stats(x, lo, T, u0, u1 - u0, slots)
        if world > 1:
            # this rank's block (a copy: the collective's input must not alias its output)
            dist.all_gather_into_tensor(slots[:world * plan.U], slots[u0:u0 + plan.U].clone(), group=self.group)
        seed = self.seed if seed is None else seed
        packed = self.wire == "packed2"
        cbytes = (plan.max_len + 15) // 16 * 16   # int8 wire: 16-B aligned records
        if self.dense == "replicated" and world > 1 and not packed:
            sendc = torch.empty(cbytes, dtype=torch.int8, device=dev)
            codes = sendc[:hi - lo]
        else:
            codes = torch.empty(hi - lo, dtype=torch.int8, device=dev)
        K.encode(x, lo, T, u0, u1 - u0, clip, u, seed, codes, slots)
        scalars = torch.empty(len(plan.sizes), dtype=torch.float32, device=dev)
        K.scalars(T, clip, slots, scalars)
        self.last_codes, self.last_scalars = codes, scalars
        if self.dense == "shard":
            s0, s1, own = plan.own[rank]
            if not own:
                return torch.empty(0, dtype=torch.float32, device=dev)
            return K.decode(codes, scalars[s0:s1 + 1], own, hi - lo)
        if world == 1:
            return K.decode(codes, scalars, plan.sizes, plan.n)
        # every rank's element range boundaries, for the decode through the records
        lkey = ("lo", plan.sizes, world, str(dev))
        rank_lo = self._slots.get(lkey)
        if rank_lo is None:
            rank_lo = self._slots[lkey] = torch.tensor([a for a, _ in plan.ranges] + [plan.n], dtype=torch.int64,
                                                       device=dev)
        # the decode through the records holds the segment table in LDS: up to seg_max() tensors
        direct = len(plan.sizes) <= K.seg_max() and world <= 64
        if packed:
            # every rank's block padded to the longest range's packed size (16-B multiples); the
            # padding is never read
            pb = (K.pack_bytes(plan.max_len) + 15) // 16 * 16
            send = torch.empty(pb, dtype=torch.uint8, device=dev)
            if hi > lo:
                K.pack(codes, send)
            gathered = torch.empty(world * pb, dtype=torch.uint8, device=dev)
            dist.all_gather_into_tensor(gathered, send, group=self.group)
            if direct:
                return K.decode_records(gathered, pb, world, rank_lo, True, scalars, plan.sizes, plan.n)
            full = torch.empty(plan.n, dtype=torch.int8, device=dev)
            for w, (a, b) in enumerate(plan.ranges):   # each block unpacked into its range
                if b > a:
                    K.unpack(gathered[w * pb:(w + 1) * pb], b - a, full[a:b])
            return K.decode(full, scalars, plan.sizes, plan.n)
        gathered = torch.empty(world * cbytes, dtype=torch.int8, device=dev)
        dist.all_gather_into_tensor(gathered, sendc, group=self.group)
        if direct:
            return K.decode_records(gathered, cbytes, world, rank_lo, False, scalars, plan.sizes, plan.n)
        full = torch.cat([gathered[w * cbytes:w * cbytes + (b - a)]
                          for w, (a, b) in enumerate(plan.ranges) if b > a])
        return K.decode(full, scalars, plan.sizes, plan.n)
