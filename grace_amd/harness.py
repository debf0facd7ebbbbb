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
    """One flat f32 buffer holding every parameter's gradient (parameters' .grad become views).
    Autograd accumulates into the existing .grad views in place, so a backward pass writes straight
    into ``flat``; clear it with ``zero_()`` (not ``optimizer.zero_grad()``, whose default
    set_to_none=True would detach the views)."""

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

    def zero_(self):
        self.flat.zero_()
        return self


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


class _ConvBN(torch.nn.Sequential):
    def __init__(self, c_in, c_out):
        super().__init__(torch.nn.Conv2d(c_in, c_out, 3, padding=1, bias=False), torch.nn.BatchNorm2d(c_out),
                         torch.nn.ReLU(inplace=True))


class _Residual(torch.nn.Module):
    def __init__(self, c):
        super().__init__()
        self.res1, self.res2 = _ConvBN(c, c), _ConvBN(c, c)

    def forward(self, x):
        return x + self.res2(self.res1(x))


class ResNet9(torch.nn.Module):
    """The DAWNBench ResNet-9 of the reference's DDP example (examples/dist/CIFAR10-dawndist/
    dawn.py:26-63: prep 64, layer1 128 + residual, layer2 256, layer3 512 + residual, 4x4 max pool,
    linear 512 -> 10 without bias, output x 0.125), from torch.nn layers: a real model whose
    backward writes the gradients the harness compresses (random init; the example's CIFAR-10
    download is not available offline, so inputs are synthetic)."""

    def __init__(self, channels=(64, 128, 256, 512), weight=0.125):
        super().__init__()
        c0, c1, c2, c3 = channels
        self.prep = _ConvBN(3, c0)
        self.layer1 = torch.nn.Sequential(_ConvBN(c0, c1), torch.nn.MaxPool2d(2), _Residual(c1))
        self.layer2 = torch.nn.Sequential(_ConvBN(c1, c2), torch.nn.MaxPool2d(2))
        self.layer3 = torch.nn.Sequential(_ConvBN(c2, c3), torch.nn.MaxPool2d(2), _Residual(c3))
        self.linear = torch.nn.Linear(c3, 10, bias=False)
        self.weight = weight

    def forward(self, x):
        x = self.layer3(self.layer2(self.layer1(self.prep(x))))
        x = torch.nn.functional.max_pool2d(x, 4).flatten(1)
        return self.linear(x) * self.weight
