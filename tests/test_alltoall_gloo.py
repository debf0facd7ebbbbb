"""AllToAll two-phase compressed allreduce (grace_amd/dist/communicator/all_to_all.py) on CPU with
gloo at W = 2 and 3, with oracle-backed QSGD / TernGrad adapters plugged into the real
communicator; checked bit-for-bit against the oracle restatement of all_to_all.py (zero padding).
The reference communicator cannot run here (gloo has no list all_to_all): parity unpinned."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import grace_oracle as O


def _streams(rank, n, chunk):
    rng = np.random.default_rng(77 + rank)
    return rng.random(n, dtype=np.float32), rng.random(chunk, dtype=np.float32)


def _adapter(kind):
    from grace_amd.dist import Compressor

    class OQuant(Compressor):
        a2a_kind = kind
        bucket_size = 128
        quantum_num = 127

        def __init__(self, u1, u2):
            super().__init__()
            self.us = [u1, u2]

        def compress(self, tensor, name):
            x = tensor.numpy().ravel()
            u = self.us.pop(0)
            if kind == "qsgd":
                c, nrm = O.qsgd_compress(x, u, 127, 128)
                return [torch.from_numpy(c), torch.from_numpy(nrm)], tensor.size()
            c, sc = O.terngrad_compress(x, u)
            return [torch.from_numpy(c), torch.from_numpy(np.asarray(sc, np.float32).reshape(1))], tensor.size()

        def decompress(self, tensors, ctx):
            if kind == "qsgd":
                return torch.from_numpy(O.qsgd_decode(tensors[0].numpy(), tensors[1].numpy(), 127, 128,
                                                      ctx.numel())).view(ctx)
            return torch.from_numpy(O.terngrad_decode(tensors[0].numpy(), tensors[1].numpy())).view(ctx)

        def aggregate(self, tensors):
            return torch.from_numpy(O.python_sum([t.numpy() for t in tensors]))

    return OQuant


def _worker(rank, world, path, outdir, kind, n):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    from grace_amd.dist.communicator.all_to_all import AllToAll
    from grace_amd.dist.memory.none import NoneMemory
    unit = world * 128 if kind == "qsgd" else world
    chunk = -(-n // unit) * unit // world
    u1, u2 = _streams(rank, n, chunk)
    g = (np.random.default_rng(500 + rank).standard_normal(n) * 0.01).astype(np.float32)
    comm = AllToAll(_adapter(kind)(u1, u2), NoneMemory(), world)
    out = comm.step(torch.from_numpy(g), "w")
    np.savez(os.path.join(outdir, f"r{rank}.npz"), out=out.numpy(), g=g)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,n", [(2, "qsgd", 4099), (3, "qsgd", 1000), (2, "terngrad", 4099),
                                          (3, "terngrad", 3001)])
def test_alltoall_two_phase(world, kind, n):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, kind, n), nprocs=world, join=True)
        outs = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(world)]
    unit = world * 128 if kind == "qsgd" else world
    chunk = -(-n // unit) * unit // world
    streams = [_streams(r, n, chunk) for r in range(world)]
    exp = O.alltoall_two_phase([o["g"] for o in outs], kind, [s[0] for s in streams], [s[1] for s in streams])
    for o in outs:
        assert np.array_equal(o["out"].view(np.uint32), exp.view(np.uint32))
