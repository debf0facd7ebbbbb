"""Golden-vector generator for the grace_amd parity tests.

Runs the REFERENCE codecs (sands-lab/grace ``grace_dl.dist``, read-only at
/root/reference) on small seeded CPU inputs and stores inputs, injected
randomness and outputs as ``.npz`` fixtures next to this file.  Only this
script ever imports the reference, and only in the build container: the
fixtures are plain data (numpy arrays + manifest.json) and are what travels to
the GPU box.  Re-run with::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Randomness capture: TernGrad / QSGD draw ``torch.empty_like(x).uniform_()``
(grace_dl/dist/compressor/terngrad.py:19, qsgd.py:31) from the global CPU
generator; we seed it, let the reference draw, and record the same stream by
re-seeding and drawing ``torch.empty(n).uniform_()`` (checked equal below).
Random-k seeds with ``sum(bytes(name)) + step`` (randomk.py:27-29); PowerSGD
uses ``use_memory=True`` with a preset ``q_memory`` (powersgd.py:38-39).
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

REF = os.environ.get("GRACE_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import torch.distributed as dist  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MANIFEST = {}

SIZES = [1, 127, 128, 129, 4099, 16411]
SHAPES2D = [(64, 33), (16, 3, 3, 3)]


def g_randn(shape, seed, scale=1.0):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=gen) * scale


def special_vec():
    v = [0.0, -0.0, float("nan"), float("inf"), float("-inf"), 1e-45, -1e-45,
         3.0, -3.0, 1.5, -1.5, 2.0 ** -126, -(2.0 ** -126), 3.4e38, -3.4e38]
    return torch.tensor(v, dtype=torch.float32)


def tied_vec(n, seed):
    # many exact duplicates: randn rounded to one decimal
    return torch.round(g_randn(n, seed) * 10) / 10


def np_(t):
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy().copy()
    return np.asarray(t)


class Store:
    def __init__(self, name):
        self.name = name
        self.arrays = {}
        self.cases = []

    def add(self, case, meta, **arrays):
        meta = dict(meta)
        meta["case"] = case
        self.cases.append(meta)
        for k, v in arrays.items():
            self.arrays[f"{case}__{k}"] = np_(v)

    def save(self):
        path = os.path.join(OUT, f"{self.name}.npz")
        np.savez_compressed(path, **self.arrays)
        MANIFEST[self.name] = self.cases
        print(f"{self.name}: {len(self.cases)} cases, {os.path.getsize(path)} bytes")


def init_world1():
    if not dist.is_initialized():
        fd, path = tempfile.mkstemp()
        os.close(fd)
        dist.init_process_group("gloo", init_method=f"file://{path}", rank=0, world_size=1)


def step_capture(comm, tensor, name):
    """Communicator.step (grace_dl/dist/__init__.py:47-51) with every stage captured."""
    t = comm.memory.compensate(tensor, name)
    t_copy = t.clone()
    payload, ctx = comm.compressor.compress(t, name)
    payload_copy = [p.clone() if isinstance(p, torch.Tensor) else p for p in payload]
    comm.memory.update(t, name, comm.compressor, payload, ctx)
    out = comm.send_receive(payload, name, ctx)
    return t_copy, payload_copy, ctx, out


# --------------------------------------------------------------------------- sign family
def gen_sign():
    from grace_dl.dist.compressor.signsgd import SignSGDCompressor
    from grace_dl.dist.compressor.signum import SignumCompressor
    from grace_dl.dist.compressor.efsignsgd import EFSignSGDCompressor
    from grace_dl.dist.memory.efsignsgd import EFSignSGDMemory
    from grace_dl.dist.compressor.onebit import OneBitCompressor
    from grace_dl.torch.compressor.onebit import OneBitCompressor as OneBitFixed
    from grace_dl.dist.communicator.allgather import Allgather
    from grace_dl.dist.memory.none import NoneMemory

    st = Store("sign")
    comp = SignSGDCompressor()
    inputs = [(f"n{n}", g_randn(n, 100 + n)) for n in SIZES]
    inputs += [(f"s{'x'.join(map(str, s))}", g_randn(s, 7)) for s in SHAPES2D]
    inputs += [("special", special_vec())]
    for case, x in inputs:
        (codes,), shape = comp.compress(x, "w")
        dec = comp.decompress([codes], shape)
        others = [g_randn(x.shape, 900 + i) for i in range(3)]
        decs = [comp.decompress(comp.compress(o, "w")[0], shape) for o in others]
        agg = comp.aggregate(decs)
        st.add("signsgd_" + case, {"codec": "signsgd", "shape": list(x.shape)},
               x=x, codes=codes, dec=dec, agg_in0=others[0], agg_in1=others[1],
               agg_in2=others[2], agg=agg)
    # Allgather world 1 full step (gloo loopback), signSGD + NoneMemory
    init_world1()
    x = g_randn(4099, 5)
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
    out = comm.step(x.clone(), "w")
    st.add("signsgd_step_w1", {"codec": "signsgd", "shape": [4099]}, x=x, out=out)

    # Signum, momentum 0.9, three steps on one name
    sg = SignumCompressor(0.9)
    seq = {}
    for s in range(3):
        x = g_randn(4099, 300 + s)
        (codes,), shape = sg.compress(x, "w")
        seq[f"x{s}"] = x
        seq[f"codes{s}"] = codes
        seq[f"mom{s}"] = sg.momentums["w"].clone()
        seq[f"dec{s}"] = sg.decompress([codes], shape)
    st.add("signum_seq", {"codec": "signum", "momentum": 0.9, "steps": 3}, **seq)

    # EF-signSGD compressor + memory, lr 0.1, three steps (compensate/compress/update)
    lr = 0.1
    ef = EFSignSGDCompressor(lr)
    mem = EFSignSGDMemory(lr)
    seq = {}
    for s in range(3):
        x = g_randn(4099, 400 + s)
        t = mem.compensate(x, "w")
        (mean, codes), shape = ef.compress(t, "w")
        mem.update(t, "w", ef, (mean, codes), shape)
        seq[f"x{s}"] = x
        seq[f"t{s}"] = t
        seq[f"mean{s}"] = mean.reshape(1)
        seq[f"codes{s}"] = codes
        seq[f"dec{s}"] = ef.decompress((mean, codes), shape)
        seq[f"res{s}"] = mem.residuals["w"]
    decs = [seq["dec0"], seq["dec1"], seq["dec2"]]
    seq["agg"] = ef.aggregate(decs)
    st.add("efsignsgd_seq", {"codec": "efsignsgd", "lr": lr, "steps": 3}, **seq)

    # One-bit: dist flavour (uint8 `~` quirk, onebit.py:29) and torch flavour (fixed)
    ob, obf = OneBitCompressor(), OneBitFixed()
    for case, x in [("n4099", g_randn(4099, 11)), ("n129", g_randn(129, 12)),
                    ("allpos", g_randn(300, 13).abs()), ("allneg", -g_randn(300, 14).abs())]:
        (mask0, mean0, mean1), shape = ob.compress(x, "w")
        dec_quirk = ob.decompress((mask0, mean0, mean1), shape)
        (m0f, mean0f, mean1f), shapef = obf.compress(x, "w")
        dec_fixed = obf.decompress((m0f, mean0f, mean1f), shapef)
        st.add("onebit_" + case, {"codec": "onebit"}, x=x, mask0=mask0,
               mean0=torch.as_tensor(mean0).reshape(1), mean1=torch.as_tensor(mean1).reshape(1),
               dec_quirk=dec_quirk, dec_fixed=dec_fixed)
    st.save()


# --------------------------------------------------------------------------- sparsifiers
def gen_sparse():
    from grace_dl.dist.compressor.topk import TopKCompressor
    from grace_dl.dist.compressor.randomk import RandomKCompressor
    from grace_dl.dist.compressor.threshold import ThresholdCompressor
    from grace_dl.dist.memory.residual import ResidualMemory
    from grace_dl.dist.communicator.allgather import Allgather
    from grace_dl.dist.communicator.allreduce import Allreduce

    init_world1()
    st = Store("sparse")
    # ---- top-k single shots
    inputs = [(f"n{n}", g_randn(n, 500 + n)) for n in SIZES]
    inputs += [(f"s{'x'.join(map(str, s))}", g_randn(s, 8)) for s in SHAPES2D]
    inputs += [("ties", tied_vec(4099, 21)), ("zeros", torch.zeros(1000)),
               ("nan", torch.cat([g_randn(200, 22), torch.tensor([float("nan"), float("inf"), -float("inf")])]))]
    for case, x in inputs:
        for ratio in (0.01, 0.1, 0.3):
            comp = TopKCompressor(ratio)
            (vals, idx), ctx = comp.compress(x, "w")
            dec = comp.decompress([vals, idx], ctx)
            st.add(f"topk_{case}_r{ratio}", {"codec": "topk", "ratio": ratio, "shape": list(x.shape)},
                   x=x, vals=vals, idx=idx, dec=dec)
    # ---- top-k + residual memory, three Allgather(world 1) steps
    for n, ratio in ((4099, 0.01), (16411, 0.01), (16411, 0.001)):
        comm = Allgather(TopKCompressor(ratio), ResidualMemory(), 1)
        seq = {}
        for s in range(3):
            g = g_randn(n, 600 + s)
            t, payload, ctx, out = step_capture(comm, g, "bucket")
            seq[f"g{s}"] = g
            seq[f"t{s}"] = t
            seq[f"vals{s}"] = payload[0]
            seq[f"idx{s}"] = payload[1]
            seq[f"res{s}"] = comm.memory.residuals["bucket"]
            seq[f"out{s}"] = out
        st.add(f"topk_residual_n{n}_r{ratio}", {"codec": "topk", "ratio": ratio, "steps": 3, "n": n}, **seq)

    # ---- random-k (seeded by name bytes + step), two names x two steps
    for ratio in (0.01, 0.3):
        comp = RandomKCompressor(ratio)
        for name, n in (("layer1.weight", 4099), ("fc.bias", 129)):
            for s in range(2):
                x = g_randn(n, 700 + s)
                h = sum(bytes(name, encoding="utf8"), comp.global_step)
                (vals,), ctx = comp.compress(x, name)
                idx = ctx[0]
                k = max(1, int(n * ratio))
                torch.manual_seed(h)
                idx_again = torch.randint(n, [k])
                assert torch.equal(idx, idx_again)
                dec = comp.decompress([vals], ctx)
                st.add(f"randomk_{name}_r{ratio}_s{s}",
                       {"codec": "randomk", "ratio": ratio, "name": name, "seed": int(h), "step": s,
                        "n": n}, x=x, vals=vals, idx=idx, dec=dec)
    # random-k through Allreduce at world 1 (payload is linear)
    comm = Allreduce(RandomKCompressor(0.1), ResidualMemory(), 1)
    seq = {}
    for s in range(2):
        g = g_randn(4099, 750 + s)
        h = sum(bytes("w", encoding="utf8"), comm.compressor.global_step)
        t, payload, ctx, out = step_capture(comm, g, "w")
        seq[f"g{s}"], seq[f"t{s}"], seq[f"idx{s}"], seq[f"vals{s}"] = g, t, ctx[0], payload[0]
        seq[f"res{s}"], seq[f"out{s}"] = comm.memory.residuals["w"], out
        seq[f"seed{s}"] = torch.tensor([h])
    st.add("randomk_residual_allreduce", {"codec": "randomk", "ratio": 0.1, "steps": 2, "n": 4099}, **seq)

    # ---- threshold
    inputs = [(f"n{n}", g_randn(n, 800 + n)) for n in (1, 129, 4099, 16411)]
    inputs += [("negonly", -g_randn(4099, 31).abs()), ("ties", tied_vec(4099, 32)),
               ("s64x33", g_randn((64, 33), 33))]
    for case, x in inputs:
        for thr in (0.01, 0.5, 100.0):
            comp = ThresholdCompressor(thr)
            (vals, idx), ctx = comp.compress(x, "w")
            dec = comp.decompress([vals, idx], ctx)
            st.add(f"threshold_{case}_t{thr}", {"codec": "threshold", "threshold": thr, "shape": list(x.shape)},
                   x=x, vals=vals, idx=idx, dec=dec)
    st.save()


# --------------------------------------------------------------------------- quantisers
def gen_quant():
    from grace_dl.dist.compressor.terngrad import TernGradCompressor
    from grace_dl.dist.compressor.qsgd import QSGDCompressor
    from grace_dl.dist.compressor.fp16 import FP16Compressor

    st = Store("quant")
    tg = TernGradCompressor()
    inputs = [(f"n{n}", g_randn(n, 1000 + n, 0.01)) for n in SIZES]
    inputs += [("s64x33", g_randn((64, 33), 9, 0.01)), ("outlier", torch.cat([g_randn(4000, 41, 0.01),
                                                                             torch.tensor([5.0, -7.0])]))]
    for case, x in inputs:
        seed = 2000 + x.numel()
        torch.manual_seed(seed)
        (codes, scalar), shape = tg.compress(x, "w")
        torch.manual_seed(seed)
        u = torch.empty(x.numel()).uniform_(0, 1)
        dec = tg.decompress((codes, scalar), shape)
        st.add(f"terngrad_{case}", {"codec": "terngrad", "seed": seed, "shape": list(x.shape)},
               x=x, u=u, codes=codes, scalar=scalar, dec=dec)

    for q, bucket in ((127, 128), (255, 128), (127, 64), (127, 512)):
        comp = QSGDCompressor(q, bucket)
        inputs = [(f"n{n}", g_randn(n, 3000 + n, 0.01)) for n in SIZES]
        xz = g_randn(1024, 51, 0.01)
        xz[128:256] = 0.0
        inputs += [("zerobucket", xz), ("s64x33", g_randn((64, 33), 10, 0.01))]
        for case, x in inputs:
            seed = 4000 + x.numel() + q
            torch.manual_seed(seed)
            (codes, norms), shape = comp.compress(x, "w")
            torch.manual_seed(seed)
            u = torch.empty(x.numel()).uniform_()
            dec = comp.decompress((codes, norms), shape)
            st.add(f"qsgd_q{q}_b{bucket}_{case}",
                   {"codec": "qsgd", "quantum_num": q, "bucket_size": bucket, "seed": seed,
                    "shape": list(x.shape)}, x=x, u=u, codes=codes, norms=norms, dec=dec)

    fp = FP16Compressor()
    for case, x in [("n4099", g_randn(4099, 61)), ("special", special_vec())]:
        (h,), dt = fp.compress(x, "w")
        st.add(f"fp16_{case}", {"codec": "fp16"}, x=x, half=h, dec=fp.decompress([h], dt))
    st.save()


# --------------------------------------------------------------------------- PowerSGD
def gen_powersgd():
    from grace_dl.dist.compressor.powersgd import PowerSGDCompressor
    from grace_dl.dist.memory.powersgd import PowerSGDMemory

    init_world1()
    st = Store("powersgd")
    for shape in ((64, 48), (33, 17), (16, 3, 3, 3), (256, 256)):
        for rank in (1, 2, 4):
            comp = PowerSGDCompressor(rank=rank, use_memory=True, world_size=1)
            x = g_randn(shape, 1100 + rank)
            n = shape[0]
            m = int(np.prod(shape[1:]))
            r = min(n, m, rank)
            q0 = g_randn((m, r), 1200 + rank)
            comp.q_memory["w"] = q0.clone()
            payload, (p, q, shp) = comp.compress(x, "w")
            dec = comp.decompress(payload, (p, q, shp))
            st.add(f"powersgd_{'x'.join(map(str, shape))}_r{rank}",
                   {"codec": "powersgd", "rank": rank, "shape": list(shape)},
                   x=x, q0=q0, p=p, q=q, dec=dec)
    # orthogonalize alone (TorchScript Gram-Schmidt, powersgd.py:7-18)
    from grace_dl.dist.compressor.powersgd import orthogonalize
    for n, r in ((4096, 4), (100, 3), (7, 1)):
        a = g_randn((n, r), 1300 + n)
        b = a.clone()
        orthogonalize(b)
        st.add(f"orth_{n}x{r}", {"codec": "orthogonalize"}, a=a, out=b)
    # ill-conditioned inputs: A = U diag(s) V^T with condition number kappa; two nearly collinear
    # columns; P = M q of a rank-2 M at r = 4 (what real low-rank gradients hand the orthogonaliser)
    for n, r, kappa in ((4096, 4, 1e4), (4096, 4, 1e7), (500, 3, 1e4)):
        gen = torch.Generator().manual_seed(1600 + int(np.log10(kappa)) + r)
        u, _ = torch.linalg.qr(torch.randn(n, r, generator=gen, dtype=torch.float64))
        v, _ = torch.linalg.qr(torch.randn(r, r, generator=gen, dtype=torch.float64))
        s = torch.logspace(0, -np.log10(kappa), r, dtype=torch.float64)
        a = (u * s) @ v.t()
        a = a.float()
        b = a.clone()
        orthogonalize(b)
        st.add(f"orth_ill_{n}x{r}_k{kappa:g}", {"codec": "orthogonalize", "kappa": kappa}, a=a, out=b)
    a = g_randn((4096, 4), 1700)
    a[:, 2] = a[:, 1] + 1e-6 * g_randn(4096, 1701)
    b = a.clone()
    orthogonalize(b)
    st.add("orth_collinear_4096x4", {"codec": "orthogonalize", "kappa": 0}, a=a, out=b)
    m2 = g_randn((4096, 2), 1702) @ g_randn((2, 1024), 1703)     # rank-2 gradient
    q = g_randn((1024, 4), 1704)
    p = torch.mm(m2, q)
    b = p.clone()
    orthogonalize(b)
    st.add("orth_rank2_4096x4", {"codec": "orthogonalize", "kappa": -1}, a=p, out=b)
    # use_memory=False path with seeded normal_ draw, plus PowerSGDMemory for two steps
    comp = PowerSGDCompressor(rank=2, use_memory=False, world_size=1)
    mem = PowerSGDMemory(comp.q_memory, compress_rank=2)
    seq = {}
    for s in range(2):
        g = g_randn((48, 40), 1400 + s)
        seed = 1500 + s
        torch.manual_seed(seed)
        t = mem.compensate(g.clone(), "w")          # draws normal (m, r) into q_memory
        qdraw_mem = comp.q_memory["w"].clone()
        payload, ctx = comp.compress(t, "w")      # draws a fresh normal (m, r) + orthogonalize
        mem.update(t, "w", comp, payload, ctx)
        torch.manual_seed(seed)
        a = torch.empty(40, 2).normal_()
        b = torch.empty(40, 2).normal_()
        assert torch.equal(a, qdraw_mem)
        seq[f"g{s}"], seq[f"t{s}"], seq[f"qdraw{s}"] = g, t, b
        seq[f"p{s}"], seq[f"q{s}"] = ctx[0], ctx[1]
        seq[f"res{s}"] = mem.residuals["w"]
        seq[f"dec{s}"] = comp.decompress(payload, ctx)
    st.add("powersgd_memory_seq", {"codec": "powersgd", "rank": 2, "steps": 2, "shape": [48, 40]}, **seq)
    st.save()


# --------------------------------------------------------------------------- world size 2 (gloo)
def _rank2_worker(rank, path, outdir):
    import torch.distributed as d
    sys.path.insert(0, REF)
    d.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=2)
    from grace_dl.dist.compressor.topk import TopKCompressor
    from grace_dl.dist.compressor.signsgd import SignSGDCompressor
    from grace_dl.dist.compressor.randomk import RandomKCompressor
    from grace_dl.dist.compressor.qsgd import QSGDCompressor
    from grace_dl.dist.compressor.terngrad import TernGradCompressor
    from grace_dl.dist.memory.residual import ResidualMemory
    from grace_dl.dist.memory.none import NoneMemory
    from grace_dl.dist.communicator.allgather import Allgather
    from grace_dl.dist.communicator.allreduce import Allreduce
    res = {}
    comm = Allgather(TopKCompressor(0.01), ResidualMemory(), 2)
    for s in range(2):
        g = g_randn(4099, 5000 + 10 * rank + s)
        t, payload, ctx, out = step_capture(comm, g, "bucket")
        res[f"topk_g{s}"], res[f"topk_vals{s}"], res[f"topk_idx{s}"] = g, payload[0], payload[1]
        res[f"topk_res{s}"], res[f"topk_out{s}"] = comm.memory.residuals["bucket"], out
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 2)
    g = g_randn(4099, 5100 + rank)
    res["sign_g"], res["sign_out"] = g, comm.step(g.clone(), "w")
    comm = Allreduce(RandomKCompressor(0.1), NoneMemory(), 2)
    g = g_randn(4099, 5200 + rank)
    t, payload, ctx, out = step_capture(comm, g, "w")
    res["randk_g"], res["randk_idx"], res["randk_out"] = g, ctx[0], out
    comm = Allgather(QSGDCompressor(127, 128), NoneMemory(), 2)
    g = g_randn(4099, 5300 + rank, 0.01)
    torch.manual_seed(5400 + rank)
    t, payload, ctx, out = step_capture(comm, g, "w")
    torch.manual_seed(5400 + rank)
    res["qsgd_g"], res["qsgd_u"] = g, torch.empty(4099).uniform_()
    res["qsgd_codes"], res["qsgd_norms"], res["qsgd_out"] = payload[0], payload[1], out
    comm = Allgather(TernGradCompressor(), NoneMemory(), 2)
    g = g_randn(4099, 5500 + rank, 0.01)
    torch.manual_seed(5600 + rank)
    t, payload, ctx, out = step_capture(comm, g, "w")
    torch.manual_seed(5600 + rank)
    res["tern_g"], res["tern_u"] = g, torch.empty(4099).uniform_()
    res["tern_codes"], res["tern_scalar"], res["tern_out"] = payload[0], payload[1], out
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **{k: np_(v) for k, v in res.items()})
    d.destroy_process_group()


def gen_dgc():
    """DGC (grace_dl/dist/compressor/dgc.py:12-50, memory/dgc.py:15-39).  The sample indices come
    from torch's global CPU generator: seeded per case and re-drawn here for the fixture."""
    from grace_dl.dist.compressor.dgc import DgcCompressor
    from grace_dl.dist.memory.dgc import DgcMemory

    init_world1()
    st = Store("dgc")
    inputs = [(f"n{n}", g_randn(n, 900 + n)) for n in (1, 129, 4099, 16411, 100003)]
    inputs += [("ties", tied_vec(4099, 41)), ("s64x33", g_randn((64, 33), 42)),
               ("nan", torch.cat([g_randn(3000, 43), torch.tensor([float("nan"), float("inf"), -float("inf")])])),
               ("zeros", torch.zeros(2000))]
    for case, x in inputs:
        for ratio in (0.01, 0.1, 0.5):
            seed = 1234 + len(st.cases)
            numel = x.numel()
            torch.manual_seed(seed)
            sidx = torch.empty([max(1, int(numel * 0.01))]).uniform_(0, numel).type(torch.long)
            comp = DgcCompressor(ratio)
            torch.manual_seed(seed)
            (vals, idx), ctx = comp.compress(x, "w")
            dec = comp.decompress([vals, idx], ctx)
            st.add(f"dgc_{case}_r{ratio}", {"codec": "dgc", "ratio": ratio, "seed": seed, "shape": list(x.shape)},
                   x=x, sample_idx=sidx, vals=vals, idx=idx, mask=ctx[1].to(torch.uint8), dec=dec)
    # DgcMemory(momentum 0.9, no clipping) + compressor, three steps (world 1)
    for n, ratio in ((4099, 0.01), (16411, 0.05)):
        comp, mem = DgcCompressor(ratio), DgcMemory(0.9, False, 1)
        seq = {}
        for s in range(3):
            g = g_randn(n, 950 + s)
            seed = 4321 + s
            seq[f"g{s}"] = g.clone()
            t = mem.compensate(g, "w")
            seq[f"t{s}"] = t.clone()
            numel = t.numel()
            torch.manual_seed(seed)
            seq[f"sidx{s}"] = torch.empty([max(1, int(numel * 0.01))]).uniform_(0, numel).type(torch.long)
            torch.manual_seed(seed)
            (vals, idx), ctx = comp.compress(t, "w")
            mem.update(t, "w", comp, (vals, idx), ctx)
            seq[f"vals{s}"], seq[f"idx{s}"] = vals, idx
            seq[f"res{s}"] = mem.residuals["w"].clone()
            seq[f"grad{s}"] = mem.gradients["w"].clone()
            seq[f"seed{s}"] = torch.tensor([seed])
        st.add(f"dgc_memory_n{n}_r{ratio}", {"codec": "dgc_memory", "ratio": ratio, "momentum": 0.9, "n": n,
                                             "steps": 3}, **seq)
    # gradient_clipping=True: dist.all_reduce returns None, so the reference raises (memory/dgc.py:17-18)
    try:
        DgcMemory(0.9, True, 1).compensate(g_randn(10, 1), "w")
        clip_raises = False
    except TypeError:
        clip_raises = True
    st.add("dgc_clipping_quirk", {"codec": "dgc_clip", "raises_type_error": clip_raises}, flag=np.array([clip_raises]))
    st.save()


def gen_torchflav():
    """The Horovod-flavour codecs whose semantics differ from grace_dl.dist (grace_dl/torch/
    compressor/{qsgd,threshold,randomk,topk,terngrad}.py).  These modules import no Horovod, so they
    run here on CPU; PowerSGD / DgcMemory / the communicators need horovod and are not pinned."""
    from grace_dl.torch.compressor.qsgd import QSGDCompressor
    from grace_dl.torch.compressor.threshold import ThresholdCompressor
    from grace_dl.torch.compressor.randomk import RandomKCompressor
    from grace_dl.torch.compressor.topk import TopKCompressor
    from grace_dl.torch.compressor.terngrad import TernGradCompressor

    st = Store("torchflav")
    # QSGD: ONE norm over the whole tensor (qsgd.py:12-31), no buckets
    for q in (127, 255):
        comp = QSGDCompressor(q)
        inputs = [(f"n{n}", g_randn(n, 6000 + n, 0.01)) for n in (1, 129, 4099, 16411, 100003)]
        inputs += [("s64x33", g_randn((64, 33), 61, 0.01)), ("zeros", torch.zeros(300)),
                   ("outlier", torch.cat([g_randn(5000, 62, 0.01), torch.tensor([3.0, -4.0])]))]
        for case, x in inputs:
            seed = 7000 + x.numel() + q
            torch.manual_seed(seed)
            (codes, norm), shape = comp.compress(x, "w")
            torch.manual_seed(seed)
            u = torch.empty(x.numel()).uniform_()
            dec = comp.decompress((codes, norm), shape)
            st.add(f"qsgd_q{q}_{case}", {"codec": "qsgd", "quantum_num": q, "seed": seed, "shape": list(x.shape)},
                   x=x, u=u, codes=codes, norm=norm.reshape(1), dec=dec)
    # threshold: strict |x| > thr, int64 indices, ctx (shape, numel) (threshold.py:12-27)
    inputs = [(f"n{n}", g_randn(n, 6100 + n)) for n in (1, 129, 4099, 16411)]
    inputs += [("ties", tied_vec(4099, 63)), ("special", special_vec()), ("s64x33", g_randn((64, 33), 64))]
    for case, x in inputs:
        for thr in (0.01, 0.5, 1.5, 100.0):
            comp = ThresholdCompressor(thr)
            (vals, idx), ctx = comp.compress(x, "w")
            dec = comp.decompress([vals, idx], ctx)
            st.add(f"threshold_{case}_t{thr}", {"codec": "threshold", "threshold": thr, "shape": list(x.shape)},
                   x=x, vals=vals, idx=idx, dec=dec)
    # random-k: randperm(numel)[:k] without replacement, seeded sum(bytes(name)) + step (randomk.py:6-34)
    for ratio in (0.01, 0.3):
        comp = RandomKCompressor(ratio)
        for name, n in (("layer1.weight", 4099), ("fc.bias", 129), ("conv.w", 100003)):
            for s in range(2):
                x = g_randn(n, 6200 + s)
                h = sum(bytes(name, encoding="utf8"), comp.global_step)
                (vals,), ctx = comp.compress(x, name)
                dec = comp.decompress([vals], ctx)
                st.add(f"randomk_{name}_r{ratio}_s{s}",
                       {"codec": "randomk", "ratio": ratio, "name": name, "seed": int(h), "n": n},
                       x=x, vals=vals, idx=ctx[0], dec=dec)
    # top-k: int64 indices, ctx (numel, shape) (topk.py:6-36)
    inputs = [(f"n{n}", g_randn(n, 6300 + n)) for n in (1, 129, 4099, 16411)]
    inputs += [("s16x3x3x3", g_randn((16, 3, 3, 3), 65)), ("zeros", torch.zeros(1000))]
    for case, x in inputs:
        for ratio in (0.01, 0.3):
            comp = TopKCompressor(ratio)
            (vals, idx), ctx = comp.compress(x, "w")
            dec = comp.decompress([vals, idx], ctx)
            st.add(f"topk_{case}_r{ratio}", {"codec": "topk", "ratio": ratio, "shape": list(x.shape)},
                   x=x, vals=vals, idx=idx, dec=dec)
    # TernGrad: rnd = uniform_(0, scalar) instead of uniform_(0, 1) * scalar (terngrad.py:19)
    tg = TernGradCompressor()
    for case, x in [(f"n{n}", g_randn(n, 6400 + n, 0.01)) for n in (1, 129, 4099, 16411)] + \
                   [("outlier", torch.cat([g_randn(4000, 66, 0.01), torch.tensor([5.0, -7.0])]))]:
        seed = 8000 + x.numel()
        torch.manual_seed(seed)
        (codes, scalar), shape = tg.compress(x, "w")
        torch.manual_seed(seed)
        u = torch.empty(x.numel()).uniform_()
        dec = tg.decompress((codes, scalar), shape)
        st.add(f"terngrad_{case}", {"codec": "terngrad", "seed": seed, "shape": list(x.shape)},
               x=x, u=u, codes=codes, scalar=scalar, dec=dec)
    st.save()


def gen_world2():
    import torch.multiprocessing as mp
    st = Store("world2")
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "rdv")
        mp.spawn(_rank2_worker, args=(path, tmp), nprocs=2, join=True)
        for rank in range(2):
            with np.load(os.path.join(tmp, f"rank{rank}.npz")) as z:
                st.add(f"rank{rank}", {"world_size": 2, "rank": rank}, **{k: z[k] for k in z.files})
    st.save()


if __name__ == "__main__":
    torch.manual_seed(0)
    only = sys.argv[1:]          # e.g. "dgc": regenerate just those fixtures
    mpath = os.path.join(OUT, "manifest.json")
    if only and os.path.exists(mpath):
        with open(mpath) as f:
            MANIFEST.update(json.load(f))
    for name, fn in (("sign", gen_sign), ("sparse", gen_sparse), ("quant", gen_quant),
                     ("powersgd", gen_powersgd), ("world2", gen_world2), ("dgc", gen_dgc),
                     ("torchflav", gen_torchflav)):
        if not only or name in only:
            fn()
    with open(mpath, "w") as f:
        json.dump(MANIFEST, f, indent=1, sort_keys=True)
    if dist.is_initialized():
        dist.destroy_process_group()
