"""Kernel-level timing of the quantiser stages (device RNG vs injected uniforms), ResNet-50 set."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import resnet50_shapes  # noqa: E402
from grace_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
n = sum(sizes)
x = torch.randn(n, device="cuda") * 0.01
u = torch.rand(n, device="cuda")
codes, norms = ops.qsgd_compress(x, 127, 128, sizes=sizes, seed=1)
tc, ts = ops.terngrad_compress(x, sizes=sizes, seed=1)
res = {
    "qsgd_enc_rng": timeit(lambda: ops.qsgd_compress(x, 127, 128, sizes=sizes, seed=1)),
    "qsgd_enc_u": timeit(lambda: ops.qsgd_compress(x, 127, 128, sizes=sizes, u=u)),
    "qsgd_dec": timeit(lambda: ops.qsgd_decompress(codes, norms, 127, 128, n, sizes=sizes)),
    "tern_enc_rng": timeit(lambda: ops.terngrad_compress(x, sizes=sizes, seed=1)),
    "tern_enc_u": timeit(lambda: ops.terngrad_compress(x, sizes=sizes, u=u)),
    "tern_dec": timeit(lambda: ops.terngrad_decompress(tc, ts, n, sizes=sizes)),
    "copy_f32": timeit(lambda: u.copy_(x)),
}
for k, v in res.items():
    print(f"{k:14s} {v:8.1f} us")
