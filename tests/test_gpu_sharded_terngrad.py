"""Sharded TernGrad (grace_amd/dist/sharded_terngrad.py) with the NATIVE kernels: 2 and 3 processes
share cuda:0 over gloo (RCCL needs one device per rank).  Every rank's codes, every tensor's scalar
and the decoded bucket are compared bit-for-bit with the single-GPU codec on the whole bucket
(ops.terngrad_compress / terngrad_decompress, itself parity-tested against the reference in
test_gpu_quant.py / test_gpu_configs.py), with the device generator and with injected uniforms,
with and without an injected clip."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
F32 = np.float32

# tensors spanning 0..4 units of 16384, unaligned offsets, a 1-element tensor
SIZES = [64, 16384, 100003, 1, 2048, 16385, 40000, 7, 65536, 3001]


def _data(seed):
    rng = np.random.default_rng(seed)
    flat = np.concatenate([(rng.standard_normal(n) * (0.01 * (1 + i % 3))).astype(F32) for i, n in enumerate(SIZES)])
    u = rng.random(flat.size).astype(F32)
    clip = np.array([0.02 * (1 + i % 4) for i in range(len(SIZES))], dtype=F32)
    return flat, u, clip


def _worker(rank, world, path, outdir, mode):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from grace_amd.dist.sharded_terngrad import ShardedTernGrad
    dense, use_u, use_clip, wire = mode
    eng = ShardedTernGrad(dense=dense, seed=11, wire=wire)
    flat, u, clip = _data(3)
    lo, hi = eng.partition(SIZES)[rank]
    res = {"lo": np.array([lo, hi])}
    for step in range(2):   # two steps: the slot array and tables are reused
        x = torch.from_numpy(flat[lo:hi] * F32(step + 1)).cuda()
        out = eng.step(x, SIZES, clip=torch.from_numpy(clip).cuda() if use_clip else None,
                       u=torch.from_numpy(u[lo:hi]).cuda() if use_u else None)
        res[f"out{step}"] = out.cpu().numpy()
        res[f"codes{step}"] = eng.last_codes.cpu().numpy()
        res[f"scalars{step}"] = eng.last_scalars.cpu().numpy()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _bits(a, b):
    return np.array_equal(np.asarray(a, F32).view(np.uint32), np.asarray(b, F32).view(np.uint32))


@pytest.mark.parametrize("world", [2, 3])
# (dense, injected u, injected clip, wire of the code all-gather)
@pytest.mark.parametrize("mode", [("replicated", False, False, "packed2"), ("replicated", True, True, "packed2"),
                                  ("replicated", False, True, "int8"), ("shard", True, False, "packed2")])
def test_sharded_terngrad_native_matches_single_gpu(world, mode):
    from grace_amd import ops
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, os.path.join(tmp, "rdv"), tmp, mode), nprocs=world, join=True)
        outs = []
        for r in range(world):
            with np.load(os.path.join(tmp, f"r{r}.npz")) as z:
                outs.append({k: z[k] for k in z.files})
    dense, use_u, use_clip, _ = mode
    flat, u, clip = _data(3)
    for step in range(2):
        x = torch.from_numpy(flat * F32(step + 1)).cuda()
        codes, scalars = ops.terngrad_compress(x, SIZES, clip=torch.from_numpy(clip).cuda() if use_clip else None,
                                               u=torch.from_numpy(u).cuda() if use_u else None, seed=11)
        dec = ops.terngrad_decompress(codes, scalars, flat.size, SIZES).cpu().numpy()
        codes, scalars = codes.cpu().numpy(), scalars.cpu().numpy()
        assert np.array_equal(np.concatenate([o[f"codes{step}"] for o in outs]), codes), (step, mode)
        if use_u and use_clip:
            # fully determined: the reference restatement tensor by tensor, directly
            from oracle import grace_oracle as O
            xv, a = flat * F32(step + 1), 0
            oc, od, osc = [], [], []
            for i, n in enumerate(SIZES):
                c, sc = O.terngrad_compress(xv[a:a + n], u[a:a + n], clip[i])
                oc.append(c)
                od.append(O.terngrad_decode(c, sc))
                osc.append(sc[0])
                a += n
            assert np.array_equal(np.concatenate([o[f"codes{step}"] for o in outs]), np.concatenate(oc)), step
            for o in outs:
                assert _bits(o[f"scalars{step}"], np.array(osc, F32)), step
                if dense == "replicated":
                    assert _bits(o[f"out{step}"], np.concatenate(od)), step
        for o in outs:
            assert _bits(o[f"scalars{step}"], scalars), (step, mode)
        if dense == "shard":
            assert _bits(np.concatenate([o[f"out{step}"] for o in outs]), dec)
        else:
            for o in outs:
                assert _bits(o[f"out{step}"], dec), (step, mode)
    assert int(outs[0]["lo"][0]) == 0 and int(outs[-1]["lo"][1]) == flat.size
