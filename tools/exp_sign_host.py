"""Is the 4 MiB world-1 sign step host-bound?  Times 4000 back-to-back Allgather(SignSGD).step calls
(host wall clock of the submission loop alone, then with the device drained) against the kernel's
event time; prints per-call microseconds.  usage: python tools/exp_sign_host.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.dist.communicator.allgather import Allgather  # noqa: E402
from grace_amd.dist.compressor.signsgd import SignSGDCompressor  # noqa: E402
from grace_amd.dist.memory.none import NoneMemory  # noqa: E402
from grace_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 20
xs = [torch.randn(n, device=dev) for _ in range(4)]
comm = Allgather(SignSGDCompressor(), NoneMemory(), 1)
for i in range(200):
    comm.step(xs[i % 4], "w")
torch.cuda.synchronize()
N = 4000
t0 = time.perf_counter()
for i in range(N):
    comm.step(xs[i % 4], "w")
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
out = torch.empty(n, device=dev)
t3 = time.perf_counter()
for i in range(N):
    ops.launch_sign_step_w1(xs[i % 4], out)
t4 = time.perf_counter()
torch.cuda.synchronize()
t5 = time.perf_counter()
print({"step_submit_us": round((t1 - t0) / N * 1e6, 2), "step_total_us": round((t2 - t0) / N * 1e6, 2),
       "launch_only_submit_us": round((t4 - t3) / N * 1e6, 2), "launch_only_total_us": round((t5 - t3) / N * 1e6, 2)})
