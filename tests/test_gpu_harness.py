"""DDP loopback harness (grace_amd/harness.py): the per-parameter loop of
examples/dist/CIFAR10-dawndist/core.py:204-208 and the one-bucket variant, each equal to the
oracle top-k + residual step applied per tensor / to the flat bucket."""
import numpy as np
import pytest
import torch

from oracle import grace_oracle as O
from tests.golden_util import same_bits

pytestmark = pytest.mark.gpu
SHAPES = [(64, 3, 7, 7), (64,), (64,), (256, 64, 1, 1), (1000, 2048), (1000,)]


def _grads(model, seed):
    rng = np.random.default_rng(seed)
    out = []
    for p in model.parameters():
        g = rng.standard_normal(p.numel()).astype(np.float32)
        p.grad.copy_(torch.from_numpy(g).view_as(p))
        out.append(g)
    return out


def test_harness_parameter_loop_and_bucket():
    from grace_amd.dist.helper import grace_from_params
    from grace_amd.harness import GradBucket, ShapeModel, step_bucketed, step_parameters
    params = {"compressor": "topk", "compress_ratio": 0.01, "memory": "residual", "communicator": "allgather",
              "world_size": 1}
    model = ShapeModel(SHAPES, "cuda")
    bucket = GradBucket(model)
    grc = grace_from_params(params)
    res = [None] * len(SHAPES)
    for s in range(2):
        gs = _grads(model, s)
        step_parameters(model, grc)
        for j, (p, g) in enumerate(zip(model.parameters(), gs)):
            _, _, _, res[j], out = O.topk_residual_step(g, res[j], 0.01)
            assert same_bits(p.grad.detach().cpu().numpy().ravel(), out), (s, j)
    grc = grace_from_params(params)
    r = None
    for s in range(2):
        g = np.concatenate(_grads(model, 10 + s))
        step_bucketed(bucket, grc)
        _, _, _, r, out = O.topk_residual_step(g, r, 0.01)
        assert same_bits(bucket.flat.cpu().numpy(), out), s


@pytest.mark.parametrize("ratio", [0.01, 0.3])
def test_segmented_per_tensor_topk_matches_parameter_loop(ratio):
    """harness.step_segmented (all tensors in one launch sequence) == the per-parameter loop's
    semantics: per tensor k_i and residual, checked bit-exact against the per-tensor oracle over
    three steps; includes tensors smaller than a chunk, odd sizes and a constant (all-tie) tensor."""
    from grace_amd.dist.segmented import SegmentedTopK
    from grace_amd.harness import GradBucket, ShapeModel, step_segmented
    shapes = SHAPES + [(3,), (4099,), (5, 7, 3), (36864,), (1,)]
    model = ShapeModel(shapes, "cuda")
    bucket = GradBucket(model)
    eng = SegmentedTopK(ratio)
    res = [None] * len(shapes)
    for s in range(3):
        gs = _grads(model, 20 + s)
        gs[-2][:] = 0.5                                  # constant tensor: every key ties
        bucket.params[-2].grad.copy_(torch.from_numpy(gs[-2]).view_as(bucket.params[-2]))
        step_segmented(bucket, eng)
        vals, idx = eng.last_payload
        idx = idx.cpu().numpy().astype(np.int64)
        vals = vals.cpu().numpy()
        off = koff = 0
        for j, (p, g) in enumerate(zip(bucket.params, gs)):
            n = g.size
            _, v_or, i_or, res[j], out = O.topk_residual_step(g, res[j], ratio)
            assert same_bits(p.grad.detach().cpu().numpy().ravel(), out), (s, j)
            k = i_or.size
            mine = idx[koff:koff + k] - off
            order = np.argsort(mine)
            assert np.array_equal(mine[order], i_or.astype(np.int64)), (s, j)
            assert same_bits(vals[koff:koff + k][order], v_or), (s, j)
            assert same_bits(eng.residuals["bucket"].cpu().numpy()[off:off + n], res[j]), (s, j)
            off += n
            koff += k


def test_segmented_resnet50_set_full():
    """All 161 ResNet-50 tensors (25,557,032 elements) at 1 %, two steps, against the oracle."""
    import bench
    from grace_amd.dist.segmented import SegmentedTopK
    sizes = [int(np.prod(s)) for s in bench.resnet50_shapes()]
    eng = SegmentedTopK(0.01)
    rng = np.random.default_rng(7)
    res = [None] * len(sizes)
    for s in range(2):
        gs = [rng.standard_normal(n).astype(np.float32) * np.float32(0.01) for n in sizes]
        flat = torch.from_numpy(np.concatenate(gs)).cuda()
        out = eng.step(flat, sizes).cpu().numpy()
        off = 0
        for j, g in enumerate(gs):
            _, _, _, res[j], o = O.topk_residual_step(g, res[j], 0.01)
            assert same_bits(out[off:off + g.size], o), (s, j)
            off += g.size


def test_harness_real_backward_resnet9():
    """SURVEY.md §8f.1 with a real model: the DAWN example's ResNet-9 (harness.ResNet9, torch.nn
    layers) on synthetic CIFAR-shaped batches; ``loss.backward()`` writes every gradient into the
    GradBucket's .grad views, then (a) the reference's per-parameter loop
    (examples/dist/CIFAR10-dawndist/core.py:204-208, ``step_parameters``) on one copy of the model
    and (b) ``step_segmented`` on a second copy compress them.  Both must equal the per-tensor
    oracle top-k + residual step applied to the gradients autograd produced, over two iterations,
    and (b) must leave its results in the .grad views in place."""
    from grace_amd.dist.helper import grace_from_params
    from grace_amd.dist.segmented import SegmentedTopK
    from grace_amd.harness import GradBucket, ResNet9, step_parameters, step_segmented
    torch.manual_seed(0)
    m1 = ResNet9().cuda()
    m2 = ResNet9().cuda()
    m2.load_state_dict(m1.state_dict())
    b1, b2 = GradBucket(m1), GradBucket(m2)
    assert len(b1.params) == 25 and sum(b1.sizes) == 6_573_120
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                             "communicator": "allgather", "world_size": 1})
    eng = SegmentedTopK(0.01)
    gen = torch.Generator().manual_seed(3)
    res = [[None] * len(b1.params), [None] * len(b2.params)]
    for s in range(2):
        x = torch.randn(16, 3, 32, 32, generator=gen).cuda()
        y = torch.randint(0, 10, (16,), generator=gen).cuda()
        grads = []
        for m, b in ((m1, b1), (m2, b2)):
            b.zero_()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            grads.append(b.flat.cpu().numpy())
        offs = np.cumsum([0] + b2.sizes)
        for b in (b1, b2):                                       # .grad still views of the bucket
            assert all(p.grad.data_ptr() == b.flat[int(o):].data_ptr() for p, o in zip(b.params, offs))
        for g in grads:
            assert np.count_nonzero(g) > 0.9 * g.size            # autograd wrote the bucket
        step_parameters(m1, grc)
        step_segmented(b2, eng)
        for which, b in enumerate((b1, b2)):
            for j, p in enumerate(b.params):
                gj = grads[which][offs[j]:offs[j + 1]]
                _, _, _, res[which][j], out = O.topk_residual_step(gj, res[which][j], 0.01)
                assert same_bits(p.grad.detach().cpu().numpy().ravel(), out), (("loop", "segmented")[which], s, j)


def _hash32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _sample_positions(n):
    """The segment bracket's sample positions (csrc/topk.hip seg_sample_n + sample_pos)."""
    S = min(max(n // 256, 512), 2048)
    S = min(S, n // 4)
    st = n // S
    pos = []
    for sidx in range(S):
        off = (_hash32(sidx * 0x9E3779B9 + 0x5EED) * st) >> 32
        pos.append(sidx * st + off)
    return np.array(pos, dtype=np.int64)


@pytest.mark.parametrize("world", [1, 2])
def test_segmented_edge_segments(world):
    """Large segments the sampled bracket must survive, next to small ones, bit-exact per tensor
    against the oracle over three steps: an all-tie (constant) large tensor, a large tensor with
    NaN / +-inf / -0 planted, one whose 3k largest elements avoid every sampled position (the
    bracket misses: the segment's exact fallback), a mostly-zero one (k-th key 0), and segments
    starting at odd offsets.  world 2 runs the residual-only mode (no dense output) and checks the
    payload (global indices) and residual; the exchange itself is covered in test_gpu_w8.py."""
    from grace_amd.dist.segmented import SegmentedTopK
    ratio = 0.01
    sizes = [3, 40000, 5, 50001, 65536, 7, 60000, 33000, 1, 8193, 20000, 8192]
    rng = np.random.default_rng(31)
    eng = SegmentedTopK(ratio, world_size=world)
    res = [None] * len(sizes)
    miss_pos = _sample_positions(65536)
    for s in range(3):
        gs = [rng.standard_normal(n).astype(np.float32) for n in sizes]
        gs[1][:] = np.float32(0.5)                                 # all ties
        gs[3][[0, 7, 77, 777, 50000]] = [np.nan, np.inf, -np.inf, -0.0, np.nan]
        g2 = (rng.random(65536).astype(np.float32) - np.float32(0.5))
        free = np.setdiff1d(np.arange(65536), miss_pos)
        g2[free[rng.permutation(free.size)[:3 * 655]]] = np.float32(1000.0)
        gs[4] = g2                                                 # sampled bracket misses
        z = np.zeros(60000, np.float32)
        z[rng.permutation(60000)[:60]] = rng.standard_normal(60).astype(np.float32)
        gs[6] = z                                                  # mostly zeros: the k-th key is 0
        flat = torch.from_numpy(np.concatenate(gs)).cuda()
        if world == 1:
            out = eng.step(flat, sizes).cpu().numpy()
        else:                                                      # the local half of the W > 1 step
            eng.local_step(flat, sizes)
        vals, idx = (t.cpu().numpy() for t in eng.last_payload)
        idx = idx.astype(np.int64)
        rcat = eng.residuals["bucket"].cpu().numpy()
        off = koff = 0
        for j, g in enumerate(gs):
            n = g.size
            _, v_or, i_or, res[j], o = O.topk_residual_step(g, res[j], ratio)
            if world == 1:
                assert same_bits(out[off:off + n], o), (s, j)
            k = i_or.size
            mine = idx[koff:koff + k] - off
            order = np.argsort(mine)
            assert np.array_equal(mine[order], i_or.astype(np.int64)), (s, j)
            assert same_bits(vals[koff:koff + k][order], v_or), (s, j)
            assert same_bits(rcat[off:off + n], res[j]), (s, j)
            off += n
            koff += k


def test_segmented_carry_tracks_the_residual():
    """The per-tensor residual-sample carry (SegmentedTopK._carries) is used only while the residual
    is the tensor the previous step left, unmodified: an in-place edit (version counter) or a
    replaced residual invalidates it, and every step stays bit-exact against the oracle."""
    from grace_amd.dist.segmented import SegmentedTopK
    ratio = 0.01
    sizes = [1 << 20, 4099, (1 << 19) + 3, 100000, 9000]
    eng = SegmentedTopK(ratio)
    rng = np.random.default_rng(77)
    res = [None] * len(sizes)
    valid_seen = []
    for s in range(5):
        gs = [rng.standard_normal(n).astype(np.float32) for n in sizes]
        r = eng.residuals.get("bucket")
        if s == 2:
            r.mul_(2.0)                                   # in place: the carry no longer matches
            res = [x * np.float32(2.0) for x in res]
        if s == 3:
            eng.residuals["bucket"] = r.clone()           # replaced: another tensor
        if r is not None:
            T = eng.tables(sizes, r.device, True, True)
            valid_seen.append(eng._carry_for("bucket", eng.residuals["bucket"], True, T)[1])
        out = eng.step(torch.from_numpy(np.concatenate(gs)).cuda(), sizes).cpu().numpy()
        off = 0
        for j, g in enumerate(gs):
            _, _, _, res[j], o = O.topk_residual_step(g, res[j], ratio)
            assert same_bits(out[off:off + g.size], o), (s, j)
            off += g.size
    assert valid_seen == [True, False, False, True]
