"""Sharded TernGrad protocol (grace_amd/dist/sharded_terngrad.py) on CPU with gloo, W = 2 and 3.

The device calls are replaced by a numpy emulator that restates what each computes (csrc/quant.hip:
per-unit f64 partials, a tensor's scale reduced from its units' partials in unit order, the
encoder's keep test, the decode); the partition, the slot all-gather, the code exchange and the
per-rank offsets are the product's.  With the clip injected the codes and scalars are checked
against the reference restatement (oracle.terngrad_compress, terngrad.py:14-24) per tensor; without
it, against the emulator run on the whole bucket in one process.  The GPU version with the native
kernels is tests/test_gpu_sharded_terngrad.py."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O

F32 = np.float32


class OracleTernKernels:
    """numpy restatement of the sharded TernGrad device calls (test infrastructure).  A small unit
    (97 elements) so that tensors span several units and ranks."""

    UNIT = 97

    def seg_max(self):
        return 512

    def unit(self):
        return self.UNIT

    def new_slots(self, nslots, device):
        return torch.zeros((nslots, 4), dtype=torch.float64)   # sum, sum of squares, max |x|, NaN

    def tables(self, sizes, device):
        seg, sub = [0], [0]
        for n in sizes:
            seg.append(seg[-1] + n)
            sub.append(sub[-1] + (n + self.UNIT - 1) // self.UNIT)
        return seg, sub, sub[-1]

    @staticmethod
    def _unit_range(T, unit):
        seg, sub, _ = T
        s = max(i for i in range(len(seg) - 1) if sub[i] <= unit)
        a = seg[s] + (unit - sub[s]) * OracleTernKernels.UNIT
        return s, a, min(a + OracleTernKernels.UNIT, seg[s + 1])

    def stats(self, x, xoff, T, unit0, nu, slots):
        xv = x.numpy()
        for unit in range(unit0, unit0 + nu):
            _, a, b = self._unit_range(T, unit)
            v = xv[a - xoff:b - xoff].astype(np.float64)
            fin = ~np.isnan(v)
            slots[unit] = torch.tensor([v.sum(), (v * v).sum(), float(np.abs(v[fin]).max()) if fin.any() else 0.0,
                                        float((~fin).any())], dtype=torch.float64)

    @staticmethod
    def _scale(T, s, slots, clip):
        seg, sub, _ = T
        p = slots[sub[s]:sub[s + 1]].numpy()
        if clip is not None:
            c = F32(clip.numpy()[s])
        else:
            nn = float(seg[s + 1] - seg[s])
            mean = p[:, 0].sum() / nn
            var = max(p[:, 1].sum() / nn - mean * mean, 0.0)
            c = F32(2.5 * float(F32(np.sqrt(var))))
        nan = p[:, 3].any() or np.isnan(c)
        return c, (F32(np.nan) if nan else min(F32(p[:, 2].max()), c))

    def encode(self, x, xoff, T, unit0, nu, clip, u, seed, codes, slots):
        xv, uv, cv = x.numpy(), u.numpy(), codes.numpy()
        for unit in range(unit0, unit0 + nu):
            s, a, b = self._unit_range(T, unit)
            c, scalar = self._scale(T, s, slots, clip)
            xs = xv[a - xoff:b - xoff]
            cl = np.minimum(np.maximum(xs, -c), c).astype(F32)
            keep = ~((uv[a - xoff:b - xoff] * scalar).astype(F32) >= np.abs(cl))
            cv[a - xoff:b - xoff] = np.where(keep, np.sign(cl) * (scalar != 0), 0).astype(np.int8)

    def scalars(self, T, clip, slots, out):
        for s in range(len(T[0]) - 1):
            out[s] = float(self._scale(T, s, slots, clip)[1])

    def decode(self, codes, scalars, sizes, n):
        sc = np.repeat(scalars.numpy().astype(F32), sizes)
        return torch.from_numpy((codes.numpy().astype(F32) * sc).astype(F32))

    def decode_records(self, records, rec_bytes, world, rank_lo, packed, scalars, sizes, n):
        """the product's record layout read back in numpy (each rank's block at w * rec_bytes)"""
        lo = rank_lo.numpy()
        rec = records.numpy().view(np.uint8)
        parts = []
        for w in range(world):
            L = int(lo[w + 1] - lo[w])
            if L == 0:
                continue
            blk = rec[w * rec_bytes:(w + 1) * rec_bytes]
            if packed:
                parts.append(O.pack2_decode(blk[:self.pack_bytes(L)], L) - 1)
            else:
                parts.append(blk[:L].view(np.int8).astype(np.int64))
        codes = torch.from_numpy(np.concatenate(parts).astype(np.int8))
        return self.decode(codes, scalars, sizes, n)

    def pack_bytes(self, n):
        return n // 4 + 1   # packing.py pads with range(0, 4 - n % 4)

    def pack(self, codes, out):
        p = O.pack2_encode(codes.numpy().astype(np.int64) + 1)
        out[:p.size].copy_(torch.from_numpy(p))

    def unpack(self, packed, n, out):
        v = O.pack2_decode(packed.numpy()[:self.pack_bytes(n)], n) - 1
        out.copy_(torch.from_numpy(v.astype(np.int8)))


def _bucket(sizes, seed):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal(n) * (0.01 * (i + 1))).astype(F32) for i, n in enumerate(sizes)]


def _worker(rank, world, path, outdir, sizes, dense, use_clip, wire="packed2"):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.sharded_terngrad import ShardedTernGrad
    eng = ShardedTernGrad(dense=dense, kernels=OracleTernKernels(), wire=wire)
    flat = np.concatenate(_bucket(sizes, 7))
    u = np.random.default_rng(8).random(flat.size).astype(F32)
    clip = torch.from_numpy(np.array([0.015 * (i + 1) for i in range(len(sizes))], dtype=F32)) if use_clip else None
    lo, hi = eng.partition(sizes)[rank]
    out = eng.step(torch.from_numpy(flat[lo:hi].copy()), sizes, clip=clip, u=torch.from_numpy(u[lo:hi].copy()))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), out=out.numpy(), codes=eng.last_codes.numpy(),
             scalars=eng.last_scalars.numpy(), lo=np.array([lo, hi]))
    dist.destroy_process_group()


def _run(world, sizes, dense, use_clip, wire="packed2"):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, sizes, dense, use_clip, wire), nprocs=world,
                 join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    return outs


def _single(sizes, use_clip):
    """The emulator on the whole bucket in one process (world 1)."""
    from grace_amd.dist.sharded_terngrad import ShardedTernGrad
    eng = ShardedTernGrad(kernels=OracleTernKernels())
    flat = np.concatenate(_bucket(sizes, 7))
    u = np.random.default_rng(8).random(flat.size).astype(F32)
    clip = torch.from_numpy(np.array([0.015 * (i + 1) for i in range(len(sizes))], dtype=F32)) if use_clip else None
    out = eng.step(torch.from_numpy(flat), sizes, clip=clip, u=torch.from_numpy(u))
    return out.numpy(), eng.last_codes.numpy(), eng.last_scalars.numpy(), flat, u


def _bits(a, b):
    return np.array_equal(np.asarray(a, F32).view(np.uint32), np.asarray(b, F32).view(np.uint32))


SIZES = [500, 97, 1, 1234, 96, 98, 3000, 5]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("use_clip", [True, False])
@pytest.mark.parametrize("wire", ["packed2", "int8"])
def test_sharded_terngrad_matches_single_bucket(world, use_clip, wire):
    outs = _run(world, SIZES, "replicated", use_clip, wire)
    out1, codes1, sc1, flat, u = _single(SIZES, use_clip)
    assert _bits(np.concatenate([o["codes"] for o in outs]), codes1.astype(F32))
    for o in outs:
        assert _bits(o["scalars"], sc1)
        assert _bits(o["out"], out1)
    # the partition tiles the bucket in rank order
    assert [int(o["lo"][0]) for o in outs][0] == 0 and int(outs[-1]["lo"][1]) == flat.size
    assert all(int(outs[r]["lo"][1]) == int(outs[r + 1]["lo"][0]) for r in range(world - 1))
    if use_clip:   # the reference's codewords and scalars per tensor, given u and the clip
        seg = np.cumsum([0] + SIZES)
        clip = [F32(0.015 * (i + 1)) for i in range(len(SIZES))]
        for s in range(len(SIZES)):
            c, sc = O.terngrad_compress(flat[seg[s]:seg[s + 1]], u[seg[s]:seg[s + 1]], clip=clip[s])
            assert np.array_equal(codes1[seg[s]:seg[s + 1]], c), s
            assert _bits(sc1[s:s + 1], sc)


def test_sharded_terngrad_dense_shard_mode():
    outs = _run(2, SIZES, "shard", True)
    out1 = _single(SIZES, True)[0]
    assert _bits(np.concatenate([o["out"] for o in outs]), out1)


@pytest.mark.parametrize("wire", ["packed2", "int8"])
def test_sharded_terngrad_rank_without_units(wire):
    """Two work units over 3 ranks: the last rank holds no element, still joins both all-gathers
    (its packed block is padding only) and decodes the whole bucket."""
    sizes = [150]
    outs = _run(3, sizes, "replicated", True, wire)
    out1 = _single(sizes, True)[0]
    assert int(outs[-1]["lo"][0]) == int(outs[-1]["lo"][1])
    for o in outs:
        assert _bits(o["out"], out1)


def test_pack2_wire_of_ternary_codes_round_trips():
    """The emulator's wire (packing.py layout of code + 1) is lossless for every length mod 4."""
    k = OracleTernKernels()
    rng = np.random.default_rng(3)
    for n in (1, 2, 3, 4, 5, 97, 1000):
        c = torch.from_numpy(rng.integers(-1, 2, n).astype(np.int8))
        buf = torch.zeros(k.pack_bytes(n) + 16, dtype=torch.uint8)
        k.pack(c, buf)
        out = torch.empty(n, dtype=torch.int8)
        k.unpack(buf, n, out)
        assert torch.equal(out, c), n
