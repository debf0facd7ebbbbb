"""Write-only 256 MiB streams: ops.fill (grace_fill) and torch's own zero_ on 3 rotated buffers,
event-timed medians -- for the A/B of non-temporal vs plain 16-B stores (libgrace_hip_plainst.so).
Usage: GRACE_HIP_LIB=... python tools/exp_write_stream.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 1 << 26
bufs = [torch.empty(n, device="cuda") for _ in range(3)]


def t(fn, reps=30):
    out = []
    for r in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(r)
        b.record()
        torch.cuda.synchronize()
        if r >= 5:
            out.append(a.elapsed_time(b) * 1e3)
    return round(statistics.median(out), 1)


res = {"lib": os.path.basename(os.environ.get("GRACE_HIP_LIB", "libgrace_hip.so")),
       "grace_fill_us": t(lambda r: ops.fill(bufs[r % 3], 0.0)),
       "torch_zero_us": t(lambda r: bufs[r % 3].zero_())}
res["grace_fill_TBps"] = round(4 * n / res["grace_fill_us"] / 1e6, 2)
print(res, flush=True)
