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
