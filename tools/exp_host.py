"""Diagnostic: host-side cost of the launch-bound 4 MiB signSGD step (bench.py --workload sign).
Times N back-to-back calls on the host (no sync inside) and the GPU-side step with events."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import _lib, ops  # noqa: E402
from grace_amd.dist.communicator.allgather import Allgather  # noqa: E402
from grace_amd.dist.compressor.signsgd import SignSGDCompressor  # noqa: E402
from grace_amd.dist.memory.none import NoneMemory  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 20
xs = [torch.randn(n, device=dev) for _ in range(64)]
out = torch.empty(n, device=dev)
comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
N = 2000


def host_us(fn):
    for i in range(50):
        fn(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(N):
        fn(i)
    h = (time.perf_counter() - t) / N * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / N * 1e6
    return round(h, 2), round(wall, 2)


s = ops._stream()
res = {
    "raw_call": host_us(lambda i: _lib.call("grace_sign_step_w1", xs[i % 64].data_ptr(), None, out.data_ptr(), n, s)),
    "raw_call+stream": host_us(lambda i: _lib.call("grace_sign_step_w1", xs[i % 64].data_ptr(), None, out.data_ptr(), n,
                                                   ops._stream())),
    "empty_like": host_us(lambda i: torch.empty_like(xs[0])),
    "ops.sign_step_w1": host_us(lambda i: ops.sign_step_w1(xs[i % 64], want_codes=False, reuse_out=True)),
    "comm.step": host_us(lambda i: comm.step(xs[i % 64], "w")),
}
print(res)
