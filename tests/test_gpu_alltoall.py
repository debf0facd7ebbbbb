"""AllToAll native decode hooks (grace_amd/dist/compressor/{qsgd,terngrad,natural}.py) on the GPU:
the one-launch phase-1 decode+sum and phase-2 decode+concat equal the per-chunk decompress +
Python-sum path of all_to_all.py bit-for-bit, and the full two-phase step matches the oracle at
world 1 with the reference's uniform stream injected."""
import numpy as np
import pytest
import torch

from grace_amd import ops
from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("kind", ["qsgd", "qsgd_cuda", "terngrad", "natural", "natural_cuda"])
@pytest.mark.parametrize("world", [2, 3])
def test_a2a_hooks_match_generic(kind, world):
    from grace_amd.dist.compressor.natural import NaturalCompressor, NaturalCompressor_CUDA
    from grace_amd.dist.compressor.qsgd import QSGDCompressor, QSGDCompressor_CUDA
    from grace_amd.dist.compressor.terngrad import TernGradCompressor
    comp = {"qsgd": QSGDCompressor(127, 128), "qsgd_cuda": QSGDCompressor_CUDA(127, 128),
            "terngrad": TernGradCompressor(), "natural": NaturalCompressor(),
            "natural_cuda": NaturalCompressor_CUDA()}[kind]
    chunk = 128 * 37
    rng = np.random.default_rng(world)
    payloads = []
    for w in range(world):
        x = torch.from_numpy((rng.standard_normal(chunk) * 0.01).astype(np.float32)).cuda()
        payloads.append(comp.compress(x, f"w{w}")[0])
    gathered = [torch.cat([p[j].reshape(-1) for p in payloads]) for j in range(len(payloads[0]))]
    shape = torch.Size([chunk])
    fast = comp.a2a_decode_sum(gathered, chunk, world)
    slow = comp.aggregate([comp.decompress(list(p), shape) for p in payloads])
    assert same_bits(_np(fast), _np(slow))
    fast = comp.a2a_decode_concat(gathered, chunk, world)
    slow = torch.cat([comp.decompress(list(p), shape) for p in payloads])
    assert same_bits(_np(fast), _np(slow))


@pytest.mark.parametrize("kind", ["qsgd", "terngrad"])
def test_a2a_world1_step_matches_oracle(kind):
    from grace_amd.dist.communicator.all_to_all import AllToAll
    from grace_amd.dist.compressor.qsgd import QSGDCompressor
    from grace_amd.dist.compressor.terngrad import TernGradCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = 4099
    comp = QSGDCompressor(127, 128, rng="torch_cpu") if kind == "qsgd" else TernGradCompressor(rng="torch_cpu")
    comm = AllToAll(comp, NoneMemory(), 1)
    g = (np.random.default_rng(3).standard_normal(n) * 0.01).astype(np.float32)
    torch.manual_seed(11)
    out = _np(comm.step(torch.from_numpy(g).cuda(), "w"))
    unit = 128 if kind == "qsgd" else 1
    chunk = -(-n // unit) * unit
    torch.manual_seed(11)
    u1 = torch.empty(n).uniform_().numpy()
    u2 = torch.empty(chunk).uniform_().numpy()
    # device norms / TernGrad scales may differ from the CPU f32 reductions by a few ulp, which can
    # flip a stochastic rounding where u sits within an ulp of the level: almost all agree
    exp = O.alltoall_two_phase([g], kind, [u1], [u2])
    close = np.isclose(out, exp, rtol=1e-5, atol=1e-8)
    assert close.mean() > 0.999, close.mean()
