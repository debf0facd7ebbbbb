"""Would two streams over two halves of the tensor list hide the segmented step's launch boundaries?
One SegmentedTopK step over all 161 ResNet-50 tensors against two engines on two streams, each over
a contiguous part of the list (its own name, residual and carry), the second part's prep free to
run beside the first part's main pass.  The dense results must be bit-identical (every tensor's
selection is its own).  Event timing of 20 back-to-back steps, median of 8 interleaved rounds."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from grace_amd.dist.segmented import SegmentedTopK  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(torch.Size(s).numel()) for s in bench.resnet50_shapes()]
n = sum(sizes)
gs = [torch.randn(n, device=dev) for _ in range(3)]


def split_at(frac):
    acc = 0
    for i, s in enumerate(sizes):
        acc += s
        if acc >= frac * n:
            return i + 1, acc
    return len(sizes), n


class One:
    def __init__(self):
        self.e = SegmentedTopK(0.01)
        self.out = torch.empty(n, device=dev)

    def step(self, g):
        self.e.step(g, sizes, out=self.out)
        return self.out


class Two:
    def __init__(self, frac):
        self.i, self.a = split_at(frac)
        self.e1, self.e2 = SegmentedTopK(0.01), SegmentedTopK(0.01)
        self.side = torch.cuda.Stream(device=dev)
        self.out = torch.empty(n, device=dev)

    def step(self, g):
        cur = torch.cuda.current_stream(dev)
        self.side.wait_stream(cur)
        self.e1.step(g[:self.a], sizes[:self.i], out=self.out[:self.a])
        with torch.cuda.stream(self.side):
            self.e2.step(g[self.a:], sizes[self.i:], out=self.out[self.a:])
        cur.wait_stream(self.side)
        return self.out


variants = {"one": One(), "two_50": Two(0.5), "two_35": Two(0.35), "two_65": Two(0.65)}
for s in range(2):   # two steps: the second uses the residuals (and carries) of the first
    outs = {k: v.step(gs[s]).clone() for k, v in variants.items()}
    for k, o in outs.items():
        assert torch.equal(o.view(torch.int32), outs["one"].view(torch.int32)), (k, s)
res = {k: [] for k in variants}
for rnd in range(9):
    for k, v in variants.items():
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for s in range(20):
            v.step(gs[s % 3])
        b.record()
        torch.cuda.synchronize()
        if rnd:
            res[k].append(a.elapsed_time(b) / 20 * 1e3)
print({k: round(statistics.median(v), 1) for k, v in res.items()}, "us per step (median of 8 rounds)")
