"""A/B of the segmented top-k's host-side layout choices in ONE process (interleaved rounds, event
timing of 20 back-to-back ddp_segmented steps on the ResNet-50 shapes, world 1): the small-segment
limit, the order of the large segments' main-pass chunks and the per-segment residual-sample
carry (on / off).  Every variant's output is checked equal to the first one's."""
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
variants = {"carry": (8192, "index", True), "no_carry": (8192, "index", False),
            "carry_size_order": (8192, "size", True)}
if os.environ.get("AB_SEG_SMALL"):   # small-segment limit A/B (must stay <= the kernel's 8192)
    variants = {f"small{v}": (int(v), "index", True) for v in os.environ["AB_SEG_SMALL"].split(",")}
engs = {}
for name, (sm, order, carry) in variants.items():
    e = SegmentedTopK(0.01)
    e._small_max, e._order, e._use_carry = sm, order, carry
    engs[name] = e
outs = {name: e.step(gs[0], sizes) for name, e in engs.items()}
ref = next(iter(outs.values()))
for name, o in outs.items():
    assert torch.equal(o.view(torch.int32), ref.view(torch.int32)), name
res = {name: [] for name in engs}
for rnd in range(9):
    for name, e in engs.items():
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for s in range(20):
            e.step(gs[s % 3], sizes)
        b.record()
        torch.cuda.synchronize()
        if rnd:
            res[name].append(a.elapsed_time(b) / 20 * 1e3)
print({name: round(statistics.median(v), 1) for name, v in res.items()}, "us per step (median of 8 rounds)")
