"""grace_shard_select's list layout at the sizes the W = 8 tests do not reach (csrc/shard.hip, r06:
the C1 list kept in blocks of 4096 entries, one apply round per block, shard_bnd one workgroup per
block): more blocks than the 512-workgroup grid (several rounds per workgroup), a gathered entry
count that is not a whole number of blocks, a single partial block, and a cut sub-bin of more than
1024 tied entries (the last arriver's radix path).  One process plays every rank on one device:
each rank's local step writes its record slot, then each rank's select runs over all of them --
checked bit for bit against the oracle's whole-bucket top-k + residual step (TopKCompressor,
grace_dl/dist/compressor/topk.py:32-42; ResidualMemory, memory/residual.py:10-20)."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu


def _bucket(case, n, seed):
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n).astype(np.float32)
    if case == "ties":
        g[rng.random(n) < 0.7] = 0.0
    return g


@pytest.mark.parametrize("world,n,case,ratio", [
    (4, 1 << 23, "normal", 0.1),      # 3.36 M gathered entries: 820 blocks, several rounds per workgroup
    (3, 3000001, "ties", 0.4),        # k > the ~900 k non-zeros: the cut among ~2.1 M zeros, the last arriver's radix select
    (5, 50001, "normal", 0.01),       # 2,500 entries: one partial block
])
def test_shard_select_blocks(world, n, case, ratio):
    from grace_amd import ops
    dev = torch.device("cuda", 0)
    k = O.ratio_k(n, ratio)
    sizes = [n // world + (1 if r < n % world else 0) for r in range(world)]
    bases = [sum(sizes[:r]) for r in range(world)]
    cap = k
    stride = ops.shard_record_words(cap)
    tab = torch.tensor(sizes + bases, dtype=torch.int64, device=dev)
    recs = torch.full((world * stride,), -1, dtype=torch.int32, device=dev)
    for r in range(world):
        recs[r * stride] = sizes[r]
        recs[r * stride + 1:r * stride + ops.SHARD_HDR] = 0
    g = _bucket(case, n, 77 + world)
    gd = torch.from_numpy(g).to(dev)
    res = [torch.empty(sizes[r], device=dev) for r in range(world)]
    for r in range(world):
        o = r * stride + ops.SHARD_HDR
        ops.topk_residual_step_swap(gd[bases[r]:bases[r] + sizes[r]], None, False, 1.0, 1.0, min(cap, sizes[r]),
                                    res[r], payload=(None, recs[o:o + cap].view(torch.float32), recs[o + cap:o + 2 * cap]))
    st = ops.new_status_word()
    pays, outs = [], []
    for r in range(world):
        out = torch.zeros(n, device=dev)
        pay = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        ops.shard_select(recs, world, r, cap, tab, k, res[r], out, 0, pay, st)
        pays.append(pay)
        outs.append(out)
    torch.cuda.synchronize()
    assert ops.status_take(st) == 0
    _, v_or, i_or, r_or, out_or = O.topk_residual_step(g, None, ratio)
    idx = np.concatenate([p.cpu().numpy() for p in pays]).astype(np.int64)
    idx = np.sort(idx[idx >= 0])
    assert np.array_equal(idx, np.sort(i_or.astype(np.int64)))
    assert same_bits(np.concatenate([x.cpu().numpy() for x in res]), r_or)
    o0 = outs[0].cpu().numpy()
    assert same_bits(o0, out_or)
    for o in outs[1:]:
        assert torch.equal(o.view(torch.int32), outs[0].view(torch.int32))
