"""World-size-2 runs of the NATIVE fused paths on one GPU: two processes share cuda:0 over the gloo
backend (RCCL needs one device per rank; the 8-GPU RCCL run is the driver's scaling bench).
Checked bit-for-bit against the reference's world-2 golden outputs."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, path, outdir, golden_path):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.none import NoneMemory
    from grace_amd.dist.memory.residual import ResidualMemory
    with np.load(golden_path, allow_pickle=False) as z:
        gold = {k: z[k] for k in z.files}
    pre = f"rank{rank}__"
    res = {}
    comm = Allgather(TopKCompressor(0.01), ResidualMemory(), 2)     # fused native step, W = 2
    for s in range(2):
        out = comm.step(torch.from_numpy(gold[pre + f"topk_g{s}"]).cuda(), "bucket")
        res[f"topk_out{s}"] = out.cpu().numpy()
        res[f"topk_res{s}"] = comm.memory.residuals["bucket"].cpu().numpy()
    # large bucket (sampled multi-kernel path, residual mode + rank-ordered sparse aggregate)
    comm = Allgather(TopKCompressor(0.01), ResidualMemory(), 2)
    for s in range(2):
        g = np.random.default_rng(1000 * rank + s).standard_normal((1 << 20) + 7).astype(np.float32)
        res[f"big_g{s}"] = g
        res[f"big_out{s}"] = comm.step(torch.from_numpy(g).cuda(), "big").cpu().numpy()
        res[f"big_res{s}"] = comm.memory.residuals["big"].cpu().numpy()
    # the same steps with one residual buffer per name (ResidualMemory(keep_spare=False): the in-place
    # W > 1 step instead of the second buffer) -- the same results bit for bit
    comm = Allgather(TopKCompressor(0.01), ResidualMemory(keep_spare=False), 2)
    for s in range(2):
        res[f"bigip_out{s}"] = comm.step(torch.from_numpy(res[f"big_g{s}"]).cuda(), "big").cpu().numpy()
        res[f"bigip_res{s}"] = comm.memory.residuals["big"].cpu().numpy()
    # variable-size payloads: threshold + residual, one host read per step (threshold.fused_step)
    from grace_amd.dist.compressor.threshold import ThresholdCompressor
    comm = Allgather(ThresholdCompressor(1.5), ResidualMemory(), 2)
    for s in range(3):
        g = np.random.default_rng(2000 * rank + s).standard_normal(5003).astype(np.float32) * (1 + rank)
        res[f"thr_g{s}"] = g
        res[f"thr_out{s}"] = comm.step(torch.from_numpy(g).cuda(), "thr").cpu().numpy()
        res[f"thr_res{s}"] = comm.memory.residuals["thr"].cpu().numpy()
    # capacity-bounded records (the overflow step is retried exactly)
    comm = Allgather(ThresholdCompressor(1.5, exchange="capacity"), ResidualMemory(), 2)
    for s in range(4):
        sc = 3.0 if s == 2 and rank == 1 else 1.0
        g = (np.random.default_rng(3000 * rank + s).standard_normal(5003) * sc).astype(np.float32)
        res[f"cap_g{s}"] = g
        res[f"cap_out{s}"] = comm.step(torch.from_numpy(g).cuda(), "thr").cpu().numpy()
        res[f"cap_res{s}"] = comm.memory.residuals["thr"].cpu().numpy()
    res["cap_overflows"] = np.array([comm.compressor.overflows])
    comm = Allgather(SignSGDCompressor(), NoneMemory(), 2)          # native majority decode
    res["sign_out"] = comm.step(torch.from_numpy(gold[pre + "sign_g"]).cuda(), "w").cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def test_fused_topk_and_sign_world2(golden):
    from tests.golden_util import GOLDEN_DIR
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(os.path.join(tmp, "rdv"), tmp, os.path.join(GOLDEN_DIR, "world2.npz")),
                 nprocs=2, join=True)
        for rank in range(2):
            g = golden.case("world2", f"rank{rank}")
            with np.load(os.path.join(tmp, f"r{rank}.npz")) as z:
                for s in range(2):
                    assert np.array_equal(z[f"topk_out{s}"].view(np.uint32), g[f"topk_out{s}"].ravel().view(np.uint32))
                    assert np.array_equal(z[f"topk_res{s}"].view(np.uint32), g[f"topk_res{s}"].ravel().view(np.uint32))
                assert np.array_equal(z["sign_out"], g["sign_out"].ravel())
        from oracle import grace_oracle as O
        zs = [np.load(os.path.join(tmp, f"r{r}.npz")) for r in range(2)]
        res = [None, None]
        for s in range(2):
            decs = []
            for r in range(2):
                t, vals, idx, res[r], _ = O.topk_residual_step(zs[r][f"big_g{s}"], res[r], 0.01)
                decs.append(O.sparse_decode(vals, idx, t.size))
                assert np.array_equal(zs[r][f"big_res{s}"].view(np.uint32), res[r].view(np.uint32))
            exp = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
            for r in range(2):
                assert np.array_equal(zs[r][f"big_out{s}"].view(np.uint32), exp.view(np.uint32))
                assert np.array_equal(zs[r][f"bigip_out{s}"].view(np.uint32), exp.view(np.uint32)), "keep_spare=False"
                assert np.array_equal(zs[r][f"bigip_res{s}"].view(np.uint32), zs[r][f"big_res{s}"].view(np.uint32))


def test_variable_size_threshold_world2_one_read():
    """Threshold + ResidualMemory through Allgather at W = 2 with different payload sizes per rank
    (the fused one-host-read exchange): outputs and residuals bit-exact against the oracle's
    reference semantics (threshold.py:12-27, residual.py:10-20, allgather.py:15-45)."""
    from oracle import grace_oracle as O
    from tests.golden_util import GOLDEN_DIR
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(os.path.join(tmp, "rdv"), tmp, os.path.join(GOLDEN_DIR, "world2.npz")),
                 nprocs=2, join=True)
        zs = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(2)]
    for pre, steps in (("thr", 3), ("cap", 4)):
        _check_thr_sequence(O, zs, pre, steps)
    # every rank takes the same capacity decisions (the stat comes from the gathered headers)
    assert zs[0]["cap_overflows"][0] >= 1 and zs[0]["cap_overflows"][0] == zs[1]["cap_overflows"][0]


def _check_thr_sequence(O, zs, pre, steps):
    res = [None, None]
    for s in range(steps):
        decs = []
        for r in range(2):
            t = O.residual_compensate(zs[r][f"{pre}_g{s}"], res[r])
            v, i = O.threshold_select(t, 1.5)
            d = O.sparse_decode(v, i, t.size)
            res[r] = O.residual_update(t, d)
            decs.append(d)
        sizes = [int((d != 0).sum()) for d in decs]
        out = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
        for r in range(2):
            assert np.array_equal(zs[r][f"{pre}_out{s}"].view(np.uint32), out.view(np.uint32)), (pre, s, r, sizes)
            assert np.array_equal(zs[r][f"{pre}_res{s}"].view(np.uint32), res[r].view(np.uint32)), (pre, s, r)
