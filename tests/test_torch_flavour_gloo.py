"""Horovod-flavour API (grace_amd/torch: async_send / wait_receive on torch.distributed work
handles) at world 2 on CPU gloo, with the oracle-backed adapters of test_dist_gloo.py.  The
reference's grace_dl.torch needs Horovod (absent); its communicators have the dist flavour's
semantics, so they are checked against the reference's world-2 dist golden outputs."""
import os
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_dist_gloo import _adapters, _bits


def _worker(rank, path, outdir, golden_path):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=2)
    from grace_amd.torch.communicator.allgather import Allgather
    from grace_amd.torch.communicator.allreduce import Allreduce
    from grace_amd.torch.communicator.broadcast import Broadcast
    from grace_amd.torch.helper import DistributedOptimizer
    OTopK, OSign, ORandomK, OThreshold, OResidual, ONone = _adapters()
    with np.load(golden_path, allow_pickle=False) as z:
        gold = {k: z[k] for k in z.files}
    pre = f"rank{rank}__"
    res = {}
    comm = Allgather(OTopK(0.01), OResidual(), 2)
    for s in range(2):   # two gradients in flight before either is received
        h0 = comm.send_step(torch.from_numpy(gold[pre + f"topk_g{s}"]), "bucket")
        res[f"topk_out{s}"] = comm.receive_step(*h0).numpy()
        res[f"topk_res{s}"] = comm.memory.residuals["bucket"]
    comm = Allgather(OSign(), ONone(), 2)
    res["sign_out"] = comm.receive_step(*comm.send_step(torch.from_numpy(gold[pre + "sign_g"]), "w")).numpy()
    comm = Broadcast(OSign(), ONone(), 2)
    res["sign_bcast"] = comm.receive_step(*comm.send_step(torch.from_numpy(gold[pre + "sign_g"]), "w")).numpy()
    comm = Allreduce(ORandomK(0.1), ONone(), 2)
    res["randk_out"] = comm.receive_step(*comm.send_step(torch.from_numpy(gold[pre + "randk_g"]), "w")).numpy()
    # variable-size payloads through the async allgather
    x = np.random.default_rng(100 + rank).standard_normal(3000).astype(np.float32)
    comm = Allgather(OThreshold(1.0), ONone(), 2)
    res["thr_x"] = x
    res["thr_out"] = comm.receive_step(*comm.send_step(torch.from_numpy(x), "w")).numpy()
    # the optimizer wrapper: hooks send during backward, step() receives
    torch.manual_seed(0)
    model = torch.nn.Linear(8, 4)
    from grace_amd.dist.compressor.none import NoneCompressor
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                               Allreduce(NoneCompressor(), ONone(), 2), model.named_parameters())
    inp = torch.full((2, 8), float(rank + 1))
    model(inp).sum().backward()
    opt.step()
    res["w_after"] = model.weight.detach().numpy().copy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def test_torch_flavour_world2(golden):
    from tests.golden_util import GOLDEN_DIR
    from oracle import grace_oracle as O
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(os.path.join(tmp, "rdv"), tmp, os.path.join(GOLDEN_DIR, "world2.npz")),
                 nprocs=2, join=True)
        outs = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(2)]
    for rank in range(2):
        g = golden.case("world2", f"rank{rank}")
        for s in range(2):
            assert _bits(outs[rank][f"topk_out{s}"], g[f"topk_out{s}"].ravel())
            assert _bits(outs[rank][f"topk_res{s}"], g[f"topk_res{s}"].ravel())
        assert _bits(outs[rank]["sign_out"], g["sign_out"].ravel())
        assert _bits(outs[rank]["sign_bcast"], g["sign_out"].ravel())
        assert _bits(outs[rank]["randk_out"], g["randk_out"].ravel())
    xs = [outs[r]["thr_x"] for r in range(2)]
    decs = [O.sparse_decode(*O.threshold_select(x, 1.0), x.size) for x in xs]
    exp = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
    for r in range(2):
        assert _bits(outs[r]["thr_out"], exp)
    # both ranks applied the same averaged gradient
    assert np.array_equal(outs[0]["w_after"], outs[1]["w_after"])
