"""TernGrad / QSGD stage timing on the ResNet-50 set with 3 rotated buffers (MALL defeated across
steps).  The library comes from GRACE_HIP_LIB, so A/B runs interleave processes on one box:
  for L in A B A B; do GRACE_HIP_LIB=$L python tools/exp_tern_ab.py; done"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import resnet50_shapes  # noqa: E402
from grace_amd import ops  # noqa: E402

sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
n = sum(sizes)
xs = [torch.randn(n, device="cuda") * 0.01 for _ in range(3)]


def timeit(fn, reps=30):
    out = []
    for rnd in range(4):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(reps):
            fn(i)
        b.record()
        torch.cuda.synchronize()
        if rnd:
            out.append(a.elapsed_time(b) / reps * 1e3)
    return round(statistics.median(out), 1)


tc = [ops.terngrad_compress(x, sizes=sizes, seed=1) for x in xs]
qc = [ops.qsgd_compress(x, 127, 128, sizes=sizes, seed=1) for x in xs]
res = {
    "tern_enc": timeit(lambda i: ops.terngrad_compress(xs[i % 3], sizes=sizes, seed=i)),
    "tern_step": timeit(lambda i: ops.terngrad_decompress(*ops.terngrad_compress(xs[i % 3], sizes=sizes, seed=i),
                                                          n, sizes=sizes)),
    "qsgd_enc": timeit(lambda i: ops.qsgd_compress(xs[i % 3], 127, 128, sizes=sizes, seed=i)),
    "qsgd_step": timeit(lambda i: ops.qsgd_decompress(*ops.qsgd_compress(xs[i % 3], 127, 128, sizes=sizes, seed=i),
                                                      127, 128, n, sizes=sizes)),
}
print(os.path.basename(os.environ.get("GRACE_HIP_LIB", "base")), res, flush=True)
