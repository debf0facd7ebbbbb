"""DDP loopback harness: the reference's training-loop use of GRACE,
examples/dist/CIFAR10-dawndist/core.py:195-209 -- after backward, every parameter's gradient goes
through ``grc.step(grad, name)`` and is copied back before the optimizer step.

``step_parameters(model, grc)`` is that loop verbatim.  All gradients can also be viewed as ONE
flat bucket (GradBucket: allocated once, the parameters' .grad tensors become views into it):
  * ``step_segmented(bucket, engine)`` keeps the loop's semantics -- per-tensor k_i and residual --
    in one launch sequence for all tensors (grace_amd.dist.segmented.SegmentedTopK);
  * ``step_bucketed(bucket, grc)`` runs ONE grc.step over the concatenation, i.e. a single global
    top-k: a different algorithm (one k for the whole model), listed for comparison.
At ResNet-50's 161 tensors the per-parameter loop is launch-bound (most tensors are a few KB)."""
import torch


def step_parameters(model, grc):
    """core.py:204-208: for each (name, parameter): grad <- grc.step(grad, name)."""
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.data
        g.copy_(grc.step(g, name))


class GradBucket:
    """One flat f32 buffer holding every parameter's gradient (parameters' .grad become views)."""

    def __init__(self, model):
        params = [p for p in model.parameters() if p.requires_grad]
        total = sum(p.numel() for p in params)
        dev = params[0].device
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n
        self.params = params
        self.sizes = [p.numel() for p in params]


def step_segmented(bucket, engine, name="bucket"):
    """The per-parameter loop's semantics (every tensor its own k_i and residual) for all tensors in
    one launch sequence: grace_amd.dist.segmented.SegmentedTopK over the bucket's segments, the
    result written back into the .grad views in place."""
    engine.step(bucket.flat, bucket.sizes, name, out=bucket.flat)


def step_bucketed(bucket, grc, name="bucket"):
    """One grc.step over the whole flat gradient bucket; results land back in the .grad views."""
    bucket.flat.copy_(grc.step(bucket.flat, name))


class ShapeModel(torch.nn.Module):
    """Parameters of given shapes (random init), for synthetic-gradient harness runs."""

    def __init__(self, shapes, device):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s, device=device) * 0.01) for s in shapes])
