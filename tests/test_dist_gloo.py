"""World-size-2 gloo tests of the communicators (grace_amd/dist/communicator) on CPU.

The codecs are GPU-only, so the collectives, payload layout, variable-size exchange, rank-ordered
aggregation and averaging are exercised here with oracle-backed CPU compressors plugged into the
real Allgather / Allreduce / Broadcast classes, and checked against the reference's own world-2
golden outputs (tests/golden/world2.npz)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O


def _adapters():
    from grace_amd.dist import Compressor, Memory

    class OTopK(Compressor):
        def __init__(self, ratio):
            super().__init__()
            self.ratio = ratio

        def compress(self, tensor, name):
            x = tensor.numpy().ravel()
            vals, idx = O.topk_select(x, O.ratio_k(x.size, self.ratio))
            return [torch.from_numpy(vals), torch.from_numpy(idx)], tensor.size()

        def decompress(self, tensors, ctx):
            vals, idx = tensors
            return torch.from_numpy(O.sparse_decode(vals.numpy(), idx.numpy(), ctx.numel())).view(ctx)

    class OSign(Compressor):
        def __init__(self):
            super().__init__(average=False)

        def compress(self, tensor, name):
            return [torch.from_numpy(O.sign_encode(tensor.numpy()))], tensor.size()

        def decompress(self, tensors, shape):
            return torch.from_numpy(O.sign_decode(tensors[0].numpy())).view(shape)

        def aggregate(self, tensors):
            return torch.from_numpy(O.sign_aggregate([t.numpy() for t in tensors]))

    class ORandomK(Compressor):
        def __init__(self, ratio):
            super().__init__()
            self.ratio, self.global_step = ratio, 0

        def compress(self, tensor, name):
            x = tensor.numpy().ravel()
            idx, _ = O.randomk_indices(name, self.global_step, x.size, self.ratio)
            self.global_step += 1
            return [torch.from_numpy(x[idx].copy())], (idx, x.size, tensor.size())

        def decompress(self, tensors, ctx):
            idx, numel, shape = ctx
            return torch.from_numpy(O.randomk_decode(tensors[0].numpy(), idx, numel)).view(shape)

    class OThreshold(Compressor):
        def __init__(self, thr):
            super().__init__(tensors_size_are_same=False)
            self.thr = thr

        def compress(self, tensor, name):
            vals, idx = O.threshold_select(tensor.numpy(), self.thr)
            return [torch.from_numpy(vals), torch.from_numpy(idx)], tensor.size()

        def decompress(self, tensors, ctx):
            vals, idx = tensors
            return torch.from_numpy(O.sparse_decode(vals.numpy(), idx.numpy(), ctx.numel())).view(ctx)

    class OResidual(Memory):
        def __init__(self):
            self.residuals = {}

        def compensate(self, tensor, name):
            r = self.residuals.get(name)
            return tensor if r is None else torch.from_numpy(O.residual_compensate(tensor.numpy(), r))

        def update(self, tensor, name, compressor, payload, ctx):
            dec = compressor.decompress(payload, ctx)
            self.residuals[name] = O.residual_update(tensor.numpy(), dec.numpy())

    class ONone(Memory):
        def compensate(self, tensor, name):
            return tensor

    return OTopK, OSign, ORandomK, OThreshold, OResidual, ONone


def _worker(rank, path, outdir, golden_path):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=2)
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.communicator.allreduce import Allreduce
    from grace_amd.dist.communicator.broadcast import Broadcast
    OTopK, OSign, ORandomK, OThreshold, OResidual, ONone = _adapters()
    with np.load(golden_path, allow_pickle=False) as z:
        gold = {k: z[k] for k in z.files}
    pre = f"rank{rank}__"
    res = {}
    comm = Allgather(OTopK(0.01), OResidual(), 2)
    for s in range(2):
        out = comm.step(torch.from_numpy(gold[pre + f"topk_g{s}"]), "bucket")
        res[f"topk_out{s}"] = out.numpy()
        res[f"topk_res{s}"] = comm.memory.residuals["bucket"]
    comm = Allgather(OSign(), ONone(), 2)
    res["sign_out"] = comm.step(torch.from_numpy(gold[pre + "sign_g"]), "w").numpy()
    comm = Broadcast(OSign(), ONone(), 2)      # rank taken from the process group
    res["sign_bcast"] = comm.step(torch.from_numpy(gold[pre + "sign_g"]), "w").numpy()
    comm = Allreduce(ORandomK(0.1), ONone(), 2)
    res["randk_out"] = comm.step(torch.from_numpy(gold[pre + "randk_g"]), "w").numpy()
    x = np.random.default_rng(100 + rank).standard_normal(3000 + 500 * rank).astype(np.float32)
    x = x[:3000]
    comm = Allgather(OThreshold(1.0), ONone(), 2)
    res["thr_x"] = x
    res["thr_out"] = comm.step(torch.from_numpy(x), "w").numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def world2_results():
    from tests.golden_util import GOLDEN_DIR
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(os.path.join(tmp, "rdv"), tmp, os.path.join(GOLDEN_DIR, "world2.npz")),
                 nprocs=2, join=True)
        out = []
        for r in range(2):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                out.append({k: z[k] for k in z.files})
        return out


def _bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, dtype=np.float32).view(np.uint32),
                          np.ascontiguousarray(b, dtype=np.float32).view(np.uint32))


def test_allgather_topk_residual_world2(golden, world2_results):
    for rank in range(2):
        g = golden.case("world2", f"rank{rank}")
        for s in range(2):
            assert _bits(world2_results[rank][f"topk_out{s}"], g[f"topk_out{s}"].ravel())
            assert _bits(world2_results[rank][f"topk_res{s}"], g[f"topk_res{s}"].ravel())


def test_allgather_and_broadcast_sign_world2(golden, world2_results):
    for rank in range(2):
        g = golden.case("world2", f"rank{rank}")
        assert _bits(world2_results[rank]["sign_out"], g["sign_out"].ravel())
        assert _bits(world2_results[rank]["sign_bcast"], g["sign_out"].ravel())


def test_allreduce_randomk_world2(golden, world2_results):
    for rank in range(2):
        g = golden.case("world2", f"rank{rank}")
        assert _bits(world2_results[rank]["randk_out"], g["randk_out"].ravel())


def test_allgather_variable_size_threshold_world2(world2_results):
    xs = [world2_results[r]["thr_x"] for r in range(2)]
    decs = [O.sparse_decode(*O.threshold_select(x, 1.0), x.size) for x in xs]
    exp = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
    for r in range(2):
        assert _bits(world2_results[r]["thr_out"], exp)
