"""Host submission cost per step of a bench workload: the bench's own step function, enqueued
behind a long device sleep (so the queue never drains and never back-pressures), timed on the
host.  A workload whose host cost per step is near its ms_per_step is launch-bound on the host.
Usage: python3 tools/exp_host.py WORKLOAD [WORKLOAD ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

_timed = bench.timed
_host = {}


def timed(fn, steps, warmup, world, dev):
    elapsed = _timed(fn, steps, warmup, world, dev)
    n = min(steps, 100)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e8))            # ~100 ms of device time ahead of the steps
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    _host["us"] = host / n * 1e6
    return elapsed


bench.timed = timed
for wl in sys.argv[1:]:
    steps = "200" if wl not in ("topk", "topk_sharded", "sign256") else "20"
    sys.argv = ["bench.py", "--workload", wl, "--steps", steps, "--no-cpu-baseline"]
    bench.main()
    print(f"HOST {wl}: {_host.get('us', float('nan')):.1f} us per step submitted", flush=True)
