"""Sharded top-k with residual error feedback: ONE gradient bucket split into contiguous shards,
one per rank (BASELINE configs[4]: 256 MiB bucket, k = 0.1 %, 8 x MI355X).

The reference has no sharded mode -- its Allgather (grace_dl/dist/communicator/allgather.py:8-45)
runs every rank on its own full bucket, and its variable-size gather reads the payload sizes back
to the host every step (allgather.py:15-18).  Here each rank owns n/W elements and the ranks
together select exactly the single-GPU top-k of the whole bucket (TopKCompressor, topk.py:32-42,
with the single-GPU engine's tie rule: larger |t| first, lower global index first), keep the
residual of their own shard (ResidualMemory, residual.py:10-20) and decode the replicated dense
bucket (or only their own slice, ``dense="shard"``).

One collective per step and no host synchronisation (grace_amd/csrc/shard.hip):
  1. the single-GPU engine selects this shard's own top-k_loc (k_loc = min(k, m); 12 B per element:
     g, r read, r' written) straight into this rank's fixed-size record -- the global top-k is
     contained in the union of the local top-k's, so the record capacity is k and nothing about
     the other ranks has to be known first;
  2. ONE all_gather_into_tensor of the records (8k bytes per rank);
  3. grace_shard_select on every rank: the exact global cut over the gathered entries, the dense
     output (zero-filled on a side stream while 1-2 run), this rank's residual restored where the
     cut rejects one of its local picks, and its payload marks.
A degenerate shard (ties, zeros) is resolved inside the local engine's own exact fallback, so
there is no bracket-miss protocol and no capacity overflow.

The partition (every rank's shard length) is agreed on a name's first step -- one all_gather and
one host read, that step only.  Every record carries its shard length, and the select kernel
checks it against the agreed table: a rank whose shard changes size later is reported on every
rank by ``ShardPartitionError`` (never a hang, never a silent mix of partitions).  The kernels
set the bit in a pinned word of this engine, one per step parity; step N + 2 waits for step N's
select (an event: by then step N + 1 is queued, so the device never idles) and takes that word,
so every rank raises at the same step N + 2 -- step N + 1's bits, which one rank may already see
and another not, are in the other word.  The parity counts this engine's steps over all names, so
a bad step of a name that is not stepped again surfaces at the engine's next-but-one step of ANY
name -- and not at all if training ends within two steps: call ``check()`` at the end of training
or of an epoch (it waits for the device and reads both words).
``check_sizes=True`` instead agrees the partition at every step (one small all_gather and one host
read per step), so a resize is handled in the step where it happens: every rank re-plans with the
new sizes, a rank whose shard kept its size keeps its error feedback, a resized rank starts from
t = g, and the event is counted in ``resizes``.

``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator of the
same calls to run the protocol on gloo.
"""
import torch
import torch.distributed as dist

from grace_amd import ops


class ShardPartitionError(RuntimeError):
    """A rank's shard length differs from the partition agreed on the name's first step."""


class ShardRecordError(ShardPartitionError):
    """The gathered records hold fewer valid entries than k (status bit 2): a corrupt record."""


class NativeShardKernels:
    """The HIP kernels behind each protocol step (GPU tensors only)."""

    HDR = ops.SHARD_HDR

    def record_words(self, cap):
        return ops.shard_record_words(cap)

    def local_step(self, g, res, has_res, k_loc, vals, idx, res_out):
        # the new residual into a second buffer: the main pass zeroes its provisional picks at
        # once instead of the finalize zeroing every selected position (grace_topk_residual_step_swap)
        ops.topk_residual_step_swap(g, res, has_res, 1.0, 1.0, k_loc, res_out, payload=(None, vals, idx))

    select = staticmethod(ops.shard_select)
    clear = staticmethod(ops.shard_clear)

    def new_status(self, device):
        return ops.new_status_word()

    def take_status(self, st):
        return ops.status_take(st)

    def fill_zero(self, x):
        return ops.fill(x, 0.0)


class _Plan:
    """Per-name state: the agreed partition and the record buffers (one allocation each)."""

    def __init__(self, K, sizes, rank, ratio, device):
        self.sizes = list(sizes)
        self.world = len(sizes)
        self.n = sum(sizes)
        self.k = ops.ratio_k(self.n, ratio)
        self.cap = self.k                       # a rank holds at most k of the global top-k
        bases = [sum(sizes[:w]) for w in range(self.world)]
        self.base = bases[rank]
        self.tab = torch.tensor(list(sizes) + bases, dtype=torch.int64).to(device)
        self.stride = K.record_words(self.cap)
        self.recs = torch.empty(self.world * self.stride, dtype=torch.int32, device=device)
        self.pay_idx = torch.full((self.cap,), -1, dtype=torch.int32, device=device)
        self.rec = None
        self.rec_m = None
        self._sel = None                        # two alternating sel_gi lists (recycled outputs)

    def sel_buffer(self, prev, device):
        """The sel_gi list this step's select writes: never the one `prev` (the recycled output's
        list, read by this step's clear) points at."""
        if self._sel is None:
            self._sel = [torch.empty(self.world * self.cap, dtype=torch.int32, device=device) for _ in range(2)]
        return self._sel[1] if prev is self._sel[0] else self._sel[0]

    def record(self, m, device, hdr):
        """This rank's send buffer: header word 0 = m, idx -1 padding past k_loc (written once per m)."""
        if self.rec is None or self.rec_m != m:
            host = torch.full((self.stride,), -1, dtype=torch.int32)
            host[:hdr] = 0
            host[0] = m
            self.rec = host.to(device)
            self.rec_m = m
        return self.rec


class ShardedTopK:
    """Top-k (ratio) + residual memory over one bucket sharded across the ranks of `group`."""

    def __init__(self, compress_ratio, group=None, dense="replicated", kernels=None, check_sizes=False,
                 recycle_output=True):
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        self.compress_ratio = compress_ratio
        self.group = group
        self.dense = dense
        self.check_sizes = check_sizes
        # A step's dense output is zero except at the W * cap selected positions.  When the caller
        # dropped the previous result of the same name unmodified (ops.OutputRecycler's rules), the
        # next step takes it back and zeroes only those positions (grace_shard_clear) instead of
        # zero-filling all of it: at configs[4] a 256 MiB write per rank and step.
        self.recycle_output = recycle_output
        self._recycler = ops.OutputRecycler()
        self.k_ops = kernels or NativeShardKernels()
        self.residuals = {}
        self._plans = {}
        self._side = {}
        self._spare = {}              # name -> the residual before the current one (next step's output buffer)
        self._status = {}             # device -> (two pinned status words, their select events)
        self._nstep = 0               # steps of this engine (all names): the status word parity
        self.last_payload = None      # (vals, idx) of this rank's record: idx = global index, or -1
        self.resizes = 0              # steps that found a rank's shard resized (check_sizes=True)
        self.host_reads = 0           # host synchronisations (first step of a name; every step with check_sizes)

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def _gather_sizes(self, m, device, world):
        if world == 1:
            return [m]
        mine = torch.tensor([m], dtype=torch.int64, device=device)
        allm = torch.empty(world, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(allm, mine, group=self.group)
        self.host_reads += 1
        return [int(v) for v in allm.cpu().tolist()]

    def _plan(self, name, m, device, world, rank):
        plan = self._plans.get(name)
        if plan is None or self.check_sizes:
            sizes = self._gather_sizes(m, device, world)
            if plan is None or sizes != plan.sizes:
                if plan is not None:
                    self.resizes += 1
                    # the recycled output's selection was taken under the old partition (its base):
                    # never clear through it
                    self._recycler.drop(name)
                plan = self._plans[name] = _Plan(self.k_ops, sizes, rank, self.compress_ratio, device)
        return plan

    def _slots(self, device):
        key = str(device)
        hit = self._status.get(key)
        if hit is None:
            hit = self._status[key] = ([self.k_ops.new_status(device) for _ in range(2)], [None, None])
        return hit

    def _raise_bits(self, bits):
        if bits & 1:
            raise ShardPartitionError(
                "grace_amd ShardedTopK: a rank's shard length changed after the name's first step (status "
                f"{bits:#x}); that step mixed partitions.  Keep every rank's shard length fixed, or "
                "construct ShardedTopK(check_sizes=True) to re-agree the partition at every step")
        if bits & 2:
            raise ShardRecordError(
                f"grace_amd ShardedTopK: the gathered records held fewer valid entries than k (status {bits:#x}): "
                "a record was corrupted in transit or written by a different build")

    def _check_status(self, device):
        """The word of this step's parity, after the select of two steps ago has finished (this
        rank's event), so every rank reports a step's bits at the same later step."""
        words, events = self._slots(device)
        slot = self._nstep & 1
        if events[slot] is not None:
            events[slot].synchronize()
            events[slot] = None
        self._raise_bits(self.k_ops.take_status(words[slot]))
        return words[slot], slot

    def check(self, device=None):
        """Wait for the device and raise if any finished step mixed partitions or saw corrupt records
        (a step never blocks on its own status: it is checked two steps later)."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        words, events = self._slots(device)
        bits = 0
        for slot in range(2):
            events[slot] = None
            bits |= self.k_ops.take_status(words[slot])
        self._raise_bits(bits)

    def _spare_residual(self, name, m, device):
        ent = self._spare.pop(name, None)
        if ent is not None:
            buf, cdata, _st = ent
            # references to buf: the popped tuple, the local name, getrefcount's argument
            if (ops.REUSE_OK and buf.numel() == m and buf.device == device and ops._getrefcount(buf) == 3
                    and ops._storage_uses(cdata) == 2):
                return buf
        return torch.empty(m, dtype=torch.float32, device=device)

    def _side_stream(self, device):
        cur = torch.cuda.current_stream(device)
        side = self._side.get(cur.cuda_stream)
        if side is None:
            side = self._side[cur.cuda_stream] = torch.cuda.Stream(device=device)
        side.wait_stream(cur)
        return cur, side

    def _clear_out(self, out, out_base, prev_sel, device):
        """A recycled output: its previous step's selected positions zeroed, on the side stream."""
        cur, side = self._side_stream(device)
        with torch.cuda.stream(side):
            self.k_ops.clear(out, out_base, prev_sel)
        out.record_stream(side)
        return out, side

    def _zero_out(self, out_len, device):
        """The dense output, zero-filled on a side stream so the fill overlaps the local step and
        the exchange; the current stream waits for it only before the select."""
        K = self.k_ops
        if device.type != "cuda":
            return K.fill_zero(torch.empty(out_len, dtype=torch.float32, device=device)), None
        cur, side = self._side_stream(device)
        with torch.cuda.stream(side):
            out = torch.empty(out_len, dtype=torch.float32, device=device)
            K.fill_zero(out)
        out.record_stream(cur)
        return out, side

    def step(self, shard, name):
        K = self.k_ops
        world, rank = self._world()
        g = shard.reshape(-1)
        dev = g.device
        m = g.numel()
        status, slot = self._check_status(dev)
        plan = self._plan(name, m, dev, world, rank)
        res = self.residuals.get(name)
        has_res = res is not None and res.numel() == m
        # this step's residual goes to a second buffer (the one the name had before the current one,
        # when nobody outside holds it): the local step reads res and writes res_new
        res_new = self._spare_residual(name, m, dev)
        if not has_res:
            res = None
        out_len = m if self.dense == "shard" else plan.n
        out_base = plan.base if self.dense == "shard" else 0
        recycle = self.recycle_output and dev.type == "cuda"
        prev_sel = None
        if recycle:
            out, prev_sel = self._recycler.take(name, (out_len, dev), alloc=False)
        if prev_sel is not None and prev_sel.numel() == plan.world * plan.cap:
            out, side = self._clear_out(out, out_base, prev_sel, dev)
        else:
            prev_sel = None
            out, side = self._zero_out(out_len, dev)
        sel = plan.sel_buffer(prev_sel, dev) if recycle else None
        rec = plan.record(m, dev, K.HDR)
        cap = plan.cap
        vals = rec[K.HDR:K.HDR + cap].view(torch.float32)
        idx = rec[K.HDR + cap:K.HDR + 2 * cap]
        K.local_step(g, res, has_res, min(cap, m), vals, idx, res_new)
        if res is not None:
            st = res.untyped_storage()
            self._spare[name] = (res, st._cdata, st)
        self.residuals[name] = res_new
        res = res_new
        if world > 1:
            dist.all_gather_into_tensor(plan.recs, rec, group=self.group)
            recs = plan.recs
        else:
            recs = rec
        if side is not None:
            torch.cuda.current_stream(dev).wait_stream(side)
        if sel is None:
            K.select(recs, world, rank, cap, plan.tab, plan.k, res, out, out_base, plan.pay_idx, status)
        else:
            K.select(recs, world, rank, cap, plan.tab, plan.k, res, out, out_base, plan.pay_idx, status, sel)
            self._recycler.keep(name, out, sel)
        if dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self._slots(dev)[1][slot] = ev
        self._nstep += 1
        self.last_payload = (vals, plan.pay_idx)
        return out
