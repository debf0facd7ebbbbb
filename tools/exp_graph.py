"""Does replaying the top-k step's three launches from a hipGraph shorten the step?  Eager vs graph
replay of ops.topk_residual_step on the 256 MiB headline bucket (3 rotated buffers, one graph each),
interleaved rounds in one process."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
gs = [torch.randn(n, device=dev) for _ in range(3)]
rs = [0.1 * torch.randn(n, device=dev) for _ in range(3)]
outs = [torch.empty(n, device=dev) for _ in range(3)]
for i in range(3):   # warm up (workspace, cached occupancy queries)
    ops.topk_residual_step(gs[i], rs[i], True, 1.0, 1.0, k, out=outs[i])
torch.cuda.synchronize()
s = torch.cuda.Stream()
graphs = []
with torch.cuda.stream(s):
    for i in range(3):
        ops.topk_residual_step(gs[i], rs[i], True, 1.0, 1.0, k, out=outs[i])
    torch.cuda.synchronize()
    for i in range(3):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            ops.topk_residual_step(gs[i], rs[i], True, 1.0, 1.0, k, out=outs[i])
        graphs.append(gr)
torch.cuda.synchronize()


def timeit(fn, reps=30):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for j in range(reps):
        fn(j)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


res = {"eager": [], "graph": []}
with torch.cuda.stream(s):
    for rnd in range(5):
        res["eager"].append(timeit(lambda j: ops.topk_residual_step(gs[j % 3], rs[j % 3], True, 1.0, 1.0, k,
                                                                    out=outs[j % 3])))
        res["graph"].append(timeit(lambda j: graphs[j % 3].replay()))
print({key: round(statistics.median(v[1:]), 1) for key, v in res.items()}, flush=True)
