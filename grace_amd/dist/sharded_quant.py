"""Sharded element-wise and bucketed quantisers: ONE bucket of tensors split over the ranks and
compressed exactly as the single-GPU codec compresses the whole bucket (SURVEY.md §8e, row
"sign / QSGD / natural: none before encode").

Codecs (the single-GPU codec each restates, and what a rank's shard must keep whole):
- ``"sign"``    SignSGDCompressor encode / decode (signsgd.py:10-22): u8 (x >= 0), decoded 2s - 1;
- ``"fp16"``    FP16Compressor (fp16.py): round-to-nearest-even cast and back;
- ``"natural"`` NaturalCompressor (natural.py:12-39), cupy flavour, device generator or injected
                randint stream;
- ``"cnat"``    NaturalCompressor_CUDA (cnat_cuda.cu:68-134), device generator, injected uniforms or
                the deterministic threshold;
- ``"qsgd"``    QSGDCompressor (qsgd.py:12-49): per tensor, buckets of ``bucket_size`` with their own
                norm, codes int8 (q < 128) or fp16.
None of them needs anything from another rank before encoding -- a QSGD bucket's norm is local to
the bucket -- so a step is: encode this rank's shard (the device generator keyed by the BUCKET's
element index, so the codes equal the whole-bucket call's: ``grace_*_compress_at``), then
``dense="replicated"``: ONE all-gather of the codes (and QSGD's bucket norms, in the same padded
record) and the decode of the whole bucket on every rank; ``dense="shard"``: the decode of this
rank's range only, no collective at all.  sign with ``wire="bits"`` (its default): the codes are
encoded straight into the 1-bit layout (grace_sign_encode_bits: word i bit j = x[32 i + j] >= 0),
an eighth of the u8 codes' bytes cross the wire, and the gathered words decode as a majority of one
(grace_sign_majority_bits, world 1: 2 b - 1) -- the same floats as the u8 path (``wire="u8"``).

Partition: QSGD by whole buckets (each tensor's buckets counted from its start, in equal contiguous
blocks per rank, as sharded TernGrad's work units); the element-wise codecs by 128-element blocks of
the flat bucket (so every shard starts on a quad of the device generator).  ``partition(sizes)``
gives every rank's [start, end) and ``step()`` takes exactly that shard.  No host synchronisation in
a step.  ``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator.
"""
import torch
import torch.distributed as dist

from grace_amd import _lib, ops

CODECS = ("sign", "fp16", "natural", "cnat", "qsgd")
_BLOCK = 128   # element-wise codecs: partition granule (a multiple of the generator's quad)


class NativeQuantKernels:
    """The HIP codec calls behind each step (GPU tensors only)."""

    def encode(self, codec, x, xoff, sizes, u, seed, q, bucket, variant, deterministic):
        """-> (codes, norms or None) of the shard x (its segment table `sizes`)."""
        if codec == "sign":
            return ops.sign_encode(x), None
        if codec == "fp16":
            return ops.fp16_compress(x), None
        if codec == "natural":
            return ops.natural_compress(x, rand_int=u, seed=seed, xoff=xoff), None
        if codec == "cnat":
            return ops.cnat_compress(x, rand=u, deterministic=deterministic, seed=seed, xoff=xoff), None
        return ops.qsgd_compress(x, q, bucket, sizes=sizes, variant=variant, u=u, seed=seed, xoff=xoff)

    def encode_into(self, codec, x, xoff, sizes, u, seed, q, bucket, variant, deterministic, codes, norms):
        """encode straight into `codes` (and QSGD's `norms`): views of this rank's send record"""
        if codec == "sign":
            ops.sign_encode(x, out=codes)
        elif codec == "fp16":
            ops.fp16_compress(x, out=codes)
        elif codec == "natural":
            ops.natural_compress(x, rand_int=u, seed=seed, xoff=xoff, out=codes)
        elif codec == "cnat":
            ops.cnat_compress(x, rand=u, deterministic=deterministic, seed=seed, xoff=xoff, out=codes)
        else:
            ops.qsgd_compress(x, q, bucket, sizes=sizes, variant=variant, u=u, seed=seed, xoff=xoff,
                              codes_out=codes, norms_out=norms)

    def seg_max(self):
        """the most tensors grace_qsgd_decompress_records takes (its segment table sits in LDS)"""
        return int(_lib.query("grace_qsgd_seg_max"))

    def decode_records(self, records, rec_bytes, norm_off, plan, rank_lo, q, variant):
        """QSGD (bucket 128): the whole bucket from the W gathered records in ONE launch
        (grace_qsgd_decompress_records), no copy into flat code / norm buffers"""
        return ops.qsgd_decompress_records(records, rec_bytes, norm_off, len(plan.ranges), plan.max_units, rank_lo,
                                           q, plan.n, sizes=list(plan.sizes), variant=variant)

    def decode(self, codec, codes, norms, sizes, n, q, bucket, variant):
        if codec == "sign":
            return ops.sign_decode(codes)
        if codec == "fp16":
            return ops.fp16_decompress(codes)
        if codec in ("natural", "cnat"):
            return ops.natural_decompress(codes, n, 0 if codec == "natural" else 1)
        return ops.qsgd_decompress(codes, norms, q, bucket, n, sizes=sizes, variant=variant)

    def encode_bits(self, x, words):
        """sign codes of x straight into the 1-bit words (ceil(n / 32) int32)"""
        _lib.call("grace_sign_encode_bits", x.data_ptr(), x.numel(), words.data_ptr(), ops._stream())

    def decode_bits(self, words, n, out):
        """n elements of 1-bit sign words -> out = 2 b - 1 (the majority of one payload)"""
        _lib.call("grace_sign_majority_bits", words.data_ptr(), 0, 1, int(n), out.data_ptr(), ops._stream())

    def code_dtype(self, codec, q):
        if codec == "fp16" or (codec == "qsgd" and q >= 128):
            return torch.float16
        return torch.int8 if codec == "qsgd" else torch.uint8


class _Plan:
    """The partition of one segment table over `world` ranks."""

    def __init__(self, codec, sizes, world, bucket):
        self.sizes = tuple(int(s) for s in sizes)
        if any(s < 1 for s in self.sizes):
            raise ValueError("ShardedQuant: empty tensor in the segment table")
        seg = [0]
        for s in self.sizes:
            seg.append(seg[-1] + s)
        self.n = seg[-1]
        self.seg = seg
        if codec == "qsgd":
            starts = []                   # global element start of every bucket
            for i, s in enumerate(self.sizes):
                starts += [seg[i] + j * bucket for j in range((s + bucket - 1) // bucket)]
        else:
            starts = list(range(0, self.n, _BLOCK))
        self.nunits = len(starts)
        starts.append(self.n)
        U = (self.nunits + world - 1) // world
        self.units = [(min(r * U, self.nunits), min((r + 1) * U, self.nunits)) for r in range(world)]
        self.ranges = [(starts[u0], starts[u1]) for u0, u1 in self.units]
        self.max_len = max(hi - lo for lo, hi in self.ranges)
        self.max_units = max(u1 - u0 for u0, u1 in self.units)
        # per rank: the parts of the tensors its range holds (QSGD's segment table of the shard)
        self.parts = []
        for lo, hi in self.ranges:
            self.parts.append([min(hi, seg[i + 1]) - max(lo, seg[i]) for i in range(len(self.sizes))
                               if seg[i] < hi and seg[i + 1] > lo])


class ShardedQuant:
    """A sign / fp16 / natural / cnat / QSGD bucket whose elements are sharded across `group`."""

    def __init__(self, codec, group=None, dense="replicated", quantum_num=127, bucket_size=128, variant=0,
                 deterministic=False, kernels=None, seed=0, wire=None):
        if codec not in CODECS:
            raise ValueError(f"codec must be one of {CODECS}")
        if wire not in (None, "bits", "u8") or (wire == "bits" and codec != "sign"):
            raise ValueError("wire: 'bits' or 'u8' for sign (default 'bits'); the other codecs send their codes as they are")
        self.bits = codec == "sign" and wire != "u8"
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        self.codec = codec
        self.group = group
        self.dense = dense
        self.q = int(quantum_num)
        self.bucket = int(bucket_size)
        self.variant = int(variant)
        self.deterministic = bool(deterministic)
        self.seed = seed
        self.k_ops = kernels or NativeQuantKernels()
        self._plans = {}
        self.last_codes = None     # this rank's codes (its element range; sign with wire="bits": int32 words)
        self.last_norms = None     # QSGD: this rank's bucket norms

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def _plan(self, sizes, world):
        key = (tuple(int(s) for s in sizes), world)
        plan = self._plans.get(key)
        if plan is None:
            plan = self._plans[key] = _Plan(self.codec, key[0], world, self.bucket)
        return plan

    def partition(self, sizes, world=None):
        """Every rank's [start, end) element range of the flat bucket."""
        return list(self._plan(sizes, world or self._world()[0]).ranges)

    def step(self, shard, sizes=None, u=None, seed=None):
        """This rank's shard (exactly partition(sizes)[rank], a tensor of its own) -> the decoded
        bucket (dense="replicated") or this rank's decoded range (dense="shard").  u: optional
        injected random stream for THIS shard's elements (natural: int32 randint draws; cnat / QSGD:
        f32 uniforms)."""
        K = self.k_ops
        world, rank = self._world()
        x = shard.reshape(-1)
        if sizes is None:
            if world != 1:
                raise ValueError("ShardedQuant: the bucket's segment sizes are needed at world > 1")
            sizes = [x.numel()]
        plan = self._plan(sizes, world)
        lo, hi = plan.ranges[rank]
        if x.numel() != hi - lo:
            raise ValueError(f"ShardedQuant: rank {rank} holds {x.numel()} elements, its range is {hi - lo} "
                             "(use partition(sizes))")
        seed = self.seed if seed is None else seed
        if self.bits:
            return self._step_bits(x, plan, world, rank, lo, hi)
        if self.dense == "replicated" and world > 1:
            return self._step_records(x, plan, world, rank, lo, hi, u, seed)
        parts = plan.parts[rank]
        if hi > lo:
            codes, norms = K.encode(self.codec, x, lo, parts, u, seed, self.q, self.bucket, self.variant,
                                    self.deterministic)
        else:
            codes = torch.empty(0, dtype=K.code_dtype(self.codec, self.q), device=x.device)
            norms = torch.empty(0, dtype=torch.float32, device=x.device) if self.codec == "qsgd" else None
        self.last_codes, self.last_norms = codes, norms
        if hi == lo:
            return torch.empty(0, dtype=torch.float32, device=x.device)
        return K.decode(self.codec, codes, norms, parts, hi - lo, self.q, self.bucket, self.variant)

    def _step_records(self, x, plan, world, rank, lo, hi, u, seed):
        """dense="replicated" at world > 1: the encoder writes this rank's codes (and QSGD's bucket
        norms) straight into its fixed-size send record, ONE all-gather moves the W records, and the
        decoder reads them through the record stride: no zero-fill, no copies.  Element-wise codecs:
        rank r's range is [r U 128, (r + 1) U 128) and the record is exactly U 128 codes (a 16-B
        multiple), so the gathered records ARE the bucket's codes in order.  QSGD: [codes (padded to
        the longest range) | norms (padded to the most buckets)], decoded in one launch through the
        records (grace_qsgd_decompress_records; bucket_size 128, other sizes copy the records back to
        flat buffers first)."""
        K = self.k_ops
        dev = x.device
        dt = K.code_dtype(self.codec, self.q)
        csz = torch.empty(0, dtype=dt).element_size()
        if self.codec != "qsgd":
            rec = torch.empty(plan.max_len, dtype=dt, device=dev)
            codes = rec[:hi - lo]
            if hi > lo:
                K.encode_into(self.codec, x, lo, plan.parts[rank], u, seed, self.q, self.bucket, self.variant,
                              self.deterministic, codes, None)
            self.last_codes, self.last_norms = codes, None
            gathered = torch.empty(world * plan.max_len, dtype=dt, device=dev)
            dist.all_gather_into_tensor(gathered, rec, group=self.group)
            return K.decode(self.codec, gathered[:plan.n], None, list(plan.sizes), plan.n, self.q, self.bucket,
                            self.variant)
        cb = (plan.max_len * csz + 15) // 16 * 16       # 16-B aligned norms and records
        nb = (plan.max_units * 4 + 15) // 16 * 16
        rec = torch.empty(cb + nb, dtype=torch.uint8, device=dev)
        u0, u1 = plan.units[rank]
        codes = rec[:(hi - lo) * csz].view(dt)
        norms = rec[cb:cb + (u1 - u0) * 4].view(torch.float32)
        if hi > lo:
            K.encode_into(self.codec, x, lo, plan.parts[rank], u, seed, self.q, self.bucket, self.variant,
                          self.deterministic, codes, norms)
        self.last_codes, self.last_norms = codes, norms
        gathered = torch.empty(world * rec.numel(), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(gathered, rec, group=self.group)
        if self.bucket == 128 and len(plan.sizes) <= K.seg_max():
            key = ("lo", plan.sizes, world, str(dev))
            rank_lo = self._plans.get(key)
            if rank_lo is None:
                rank_lo = self._plans[key] = torch.tensor([a for a, _ in plan.ranges], dtype=torch.int64, device=dev)
            return K.decode_records(gathered, rec.numel(), cb, plan, rank_lo, self.q, self.variant)
        g = gathered.view(world, -1)
        full = torch.cat([g[w, :(b - a) * csz] for w, (a, b) in enumerate(plan.ranges) if b > a]).view(dt)
        allnorms = torch.cat([g[w, cb:cb + (b - a) * 4] for w, (a, b) in enumerate(plan.units) if b > a]).view(torch.float32)
        return K.decode(self.codec, full, allnorms, list(plan.sizes), plan.n, self.q, self.bucket, self.variant)

    def _step_bits(self, x, plan, world, rank, lo, hi):
        """sign over the 1-bit wire: rank r's words are its block of the bucket's bit stream (its
        range starts on a 128-element block), padded to the longest range's words."""
        K = self.k_ops
        dev = x.device
        nw = (hi - lo + 31) // 32
        if self.dense == "shard" or world == 1:
            out = torch.empty(hi - lo, dtype=torch.float32, device=dev)
            words = torch.empty(nw, dtype=torch.int32, device=dev)
            if hi > lo:
                K.encode_bits(x, words)
                K.decode_bits(words, hi - lo, out)
            self.last_codes, self.last_norms = words, None
            return out
        per = ((plan.max_len + 31) // 32 + 3) // 4 * 4      # words per rank block, 16-B multiples
        send = torch.zeros(per, dtype=torch.int32, device=dev)
        if hi > lo:
            K.encode_bits(x, send[:nw])
        self.last_codes, self.last_norms = send[:nw], None
        gathered = torch.empty(world * per, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(gathered, send, group=self.group)
        out = torch.empty(plan.n, dtype=torch.float32, device=dev)
        if all(b - a == per * 32 for a, b in plan.ranges[:-1]):
            # every block but the last is whole: the gathered words are the bucket's bit stream
            K.decode_bits(gathered, plan.n, out)
        else:
            for w, (a, b) in enumerate(plan.ranges):
                if b > a:
                    K.decode_bits(gathered[w * per:(w + 1) * per], b - a, out[a:b])
        return out
