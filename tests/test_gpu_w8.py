"""The W > 1 paths the driver's 8-GPU run and the DDP harness execute, run natively with W ranks on
ONE GPU (the ranks share cuda:0 over gloo: RCCL needs one device per rank, and the 8-GPU RCCL run
is the driver's).  Every rank's result is checked bit-for-bit against the oracle.

1. ``Allgather(TopKCompressor(0.01), ResidualMemory(), 8).step`` on a 2^26-element (256 MiB) bucket
   for two steps: BASELINE configs[1] in the DP-replica mode ``bench.py --gpus 8`` times.  This is
   the path no smaller test reaches together: the 12-B/element main pass (no dense output at
   W > 1), ``sort_payload`` at k = 671,088, the all-gather of 8 sorted payloads and the one-pass
   8-way grouped decode (``sparse_aggregate_sorted``).  Expected: every rank's residual equals the
   oracle's step on that rank's bucket (grace_dl/dist/compressor/topk.py:32-49,
   memory/residual.py:10-20), every rank's output equals Python's rank-ordered ``sum`` of the 8
   decodes divided by 8 (grace_dl/dist/communicator/allgather.py:40-45).
2. ``SegmentedTopK(0.01, world_size=W)`` at W = 2 and 8 on the 161-tensor ResNet-50 set: the per-
   parameter DDP loop's semantics (examples/dist/CIFAR10-dawndist/core.py:203-206, every tensor its
   own k_i and residual) with one all-gather of the concatenated payloads.
3. ``grace_amd.torch.helper.DistributedOptimizer`` with the native Horovod-flavour TopK + Residual
   at W = 2, driven by a real ``loss.backward()`` through a torch.nn model, so the post-accumulate
   hooks fire ``send_step`` (grace_dl/torch/__init__.py:50-55) and ``step()`` runs ``receive_step``
   (:57-58, patch_files/horovod/torch/optimizer.py:204-237).
"""
import hashlib
import os
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
F32 = np.float32


def _progress(msg):
    """Progress on the real stderr (past pytest's capture): the W = 8 checks run for minutes."""
    sys.__stderr__.write(f"[test_gpu_w8] {msg}\n")
    sys.__stderr__.flush()


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def _init(rank, world, path):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)


# ------------------------------------------------------------------ 1. DP-replica top-k, W = 8, 2^26
N_BIG = 1 << 26


def _big_bucket(rank, step):
    return np.random.default_rng(7000 + 100 * rank + step).standard_normal(N_BIG, dtype=F32)


def _dp_worker(rank, world, path, outdir, steps):
    _init(rank, world, path)
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    assert N_BIG <= ops.SORT_PAYLOAD_MAX_N            # the sorted-payload exchange is the path taken
    comm = Allgather(TopKCompressor(0.01), ResidualMemory(), world)
    res = {}
    for s in range(steps):
        out = comm.step(torch.from_numpy(_big_bucket(rank, s)).cuda(), "bucket").cpu().numpy()
        r = comm.memory.residuals["bucket"].cpu().numpy()
        res[f"out_sha{s}"] = np.frombuffer(_digest(out).encode(), dtype=np.uint8)
        res[f"res_sha{s}"] = np.frombuffer(_digest(r).encode(), dtype=np.uint8)
        if rank == 0:
            res[f"out{s}"] = out
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_dp_replica_topk_w8_256mib():
    world, steps = 8, 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_dp_worker, args=(world, os.path.join(tmp, "rdv"), tmp, steps), nprocs=world, join=True)
        got = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                got.append({key: z[key] for key in z.files})
    res = [None] * world
    k = O.ratio_k(N_BIG, 0.01)
    assert k == 671_088
    for s in range(steps):
        acc = None                                    # Python sum: ((0 + d0) + d1) + ... in f32
        for r in range(world):
            _progress(f"dp-replica oracle step {s} rank {r}")
            _, vals, idx, res[r], _ = O.topk_residual_step(_big_bucket(r, s), res[r], 0.01)
            assert idx.size == k
            assert bytes(got[r][f"res_sha{s}"]) == _digest(res[r]).encode(), ("residual", s, r)
            d = O.sparse_decode(vals, idx, N_BIG)
            acc = (F32(0) + d) if acc is None else (acc + d)
            del d
        exp = (acc / F32(world)).astype(F32)
        assert same_bits(got[0][f"out{s}"], exp), s
        sha = _digest(exp).encode()
        assert all(bytes(g[f"out_sha{s}"]) == sha for g in got), ("output", s)


# --------------------------------------------------------- 2. segmented per-tensor top-k, W = 2 / 8
def _resnet_sizes():
    import bench
    return [int(np.prod(s)) for s in bench.resnet50_shapes()]


def _seg_grad(sizes, rank, step):
    rng = np.random.default_rng(9000 + 100 * rank + step)
    return (rng.standard_normal(sum(sizes), dtype=F32) * F32(0.01)).astype(F32)


def _seg_worker(rank, world, path, outdir, steps, sizes):
    _init(rank, world, path)
    from grace_amd.dist.segmented import SegmentedTopK
    eng = SegmentedTopK(0.01, world_size=world)
    res = {}
    for s in range(steps):
        g = torch.from_numpy(_seg_grad(sizes, rank, s)).cuda()
        out = eng.step(g, sizes, "model").cpu().numpy()
        res[f"out{s}"] = out
        res[f"res{s}"] = eng.residuals["model"].cpu().numpy()
    # in place, as harness.step_segmented runs it (out is the gradient buffer itself)
    eng2 = SegmentedTopK(0.01, world_size=world)
    g = torch.from_numpy(_seg_grad(sizes, rank, 0)).cuda()
    eng2.step(g, sizes, "model", out=g)
    res["inplace0"] = g.cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 8])
def test_segmented_topk_world(world):
    sizes = _resnet_sizes()
    assert len(sizes) == 161 and sum(sizes) == 25_557_032
    steps = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_seg_worker, args=(world, os.path.join(tmp, "rdv"), tmp, steps, sizes), nprocs=world, join=True)
        got = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(world)]
    offs = np.cumsum([0] + sizes)
    res = [[None] * len(sizes) for _ in range(world)]
    for s in range(steps):
        acc = None
        for r in range(world):
            _progress(f"segmented W={world} oracle step {s} rank {r}")
            g = _seg_grad(sizes, r, s)
            dec = np.empty_like(g)
            rr = np.empty_like(g)
            for i in range(len(sizes)):
                a, b = offs[i], offs[i + 1]
                t, vals, idx, res[r][i], _ = O.topk_residual_step(g[a:b], res[r][i], 0.01)
                dec[a:b] = O.sparse_decode(vals, idx, b - a)
                rr[a:b] = res[r][i]
            assert same_bits(got[r][f"res{s}"], rr), ("residual", world, s, r)
            acc = (F32(0) + dec) if acc is None else (acc + dec)
        exp = (acc / F32(world)).astype(F32)
        for r in range(world):
            assert same_bits(got[r][f"out{s}"], exp), ("output", world, s, r)
        if s == 0:
            for r in range(world):
                assert same_bits(got[r]["inplace0"], exp), ("in place", world, r)


# ------------------------------------------- 3. Horovod-style DistributedOptimizer, real backward
class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = torch.nn.Conv2d(3, 16, 3, padding=1, bias=False)
        self.bn1 = torch.nn.BatchNorm2d(16)
        self.conv2 = torch.nn.Conv2d(16, 32, 3, padding=1)
        self.fc = torch.nn.Linear(32 * 4 * 4, 10)

    def forward(self, x):
        x = torch.nn.functional.relu(self.bn1(self.conv1(x)))
        x = torch.nn.functional.max_pool2d(x, 2)
        x = torch.nn.functional.relu(self.conv2(x))
        x = torch.nn.functional.adaptive_avg_pool2d(x, 4)
        return self.fc(x.flatten(1))


def _opt_worker(rank, world, path, outdir, steps, ratio):
    _init(rank, world, path)
    from grace_amd.torch.communicator.allgather import Allgather
    from grace_amd.torch.compressor.topk import TopKCompressor
    from grace_amd.torch.helper import DistributedOptimizer
    from grace_amd.torch.memory.residual import ResidualMemory
    torch.manual_seed(0)                              # same initial weights on every rank
    model = _Net().cuda()
    captured = {}
    names = {p: n for n, p in model.named_parameters()}
    for p in model.parameters():                      # registered first: runs before the send hook
        p.register_post_accumulate_grad_hook(lambda q: captured.__setitem__(names[q], q.grad.detach().clone()))
    grc = Allgather(TopKCompressor(ratio), ResidualMemory(), world)
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), grc, model.named_parameters())
    gen = torch.Generator().manual_seed(100 + rank)  # each rank its own batch
    res = {}
    for s in range(steps):
        x = torch.randn(8, 3, 8, 8, generator=gen).cuda()
        y = torch.randint(0, 10, (8,), generator=gen).cuda()
        opt.zero_grad()
        captured.clear()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()                               # hooks: send_step per parameter
        assert len(opt._pending) == len(list(model.parameters()))
        opt.step()                                    # receive_step per parameter, then SGD
        for n, p in model.named_parameters():
            res[f"g{s}/{n}"] = captured[n].cpu().numpy()
            res[f"out{s}/{n}"] = p.grad.detach().cpu().numpy()
            res[f"res{s}/{n}"] = grc.memory.residuals[n].cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_distributed_optimizer_native_topk_world2_real_backward():
    world, steps, ratio = 2, 2, 0.05
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_opt_worker, args=(world, os.path.join(tmp, "rdv"), tmp, steps, ratio), nprocs=world, join=True)
        got = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(world)]
    names = sorted({key.split("/", 1)[1] for key in got[0] if key.startswith("g0/")})
    assert len(names) == 7
    res = {(r, n): None for r in range(world) for n in names}
    for s in range(steps):
        for n in names:
            decs = []
            for r in range(world):
                g = got[r][f"g{s}/{n}"]
                assert np.any(g != 0), (s, n, r)      # autograd really wrote this gradient
                t, vals, idx, res[(r, n)], _ = O.topk_residual_step(g.ravel(), res[(r, n)], ratio)
                decs.append(O.sparse_decode(vals, idx, t.size))
                assert same_bits(got[r][f"res{s}/{n}"].ravel(), res[(r, n)]), ("residual", s, n, r)
            exp = (O.python_sum(decs) / F32(world)).astype(F32)
            for r in range(world):
                assert same_bits(got[r][f"out{s}/{n}"].ravel(), exp), ("grad", s, n, r)
