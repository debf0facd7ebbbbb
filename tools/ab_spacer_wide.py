"""Wide spacer sweep (0-64 GiB) of tools/ab_spacer.py: are fitting residual / output pairs on a GPU where the 0-12 GiB range had none further apart?
(tools/ab_place5.py's fast pairs were 5-7 and 17-19 GB of allocations apart, slow ones 1.75-3.5 and
9-14 GB.)  For spacers S between the residual candidates and the output candidates, the streaming
probe's microseconds of all 4 x 3 pairs (ops.pick_pair's probe), twice per S, in one process.
usage: python tools/ab_spacer.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import _lib, ops  # noqa: E402

n = 64 * 1024 * 1024
dev = torch.device("cuda", 0)
g = torch.randn(n, device=dev)
ws = torch.zeros(int(_lib.query("grace_topk_stream_probe_workspace_bytes", n)), dtype=torch.uint8, device=dev)


def probe(r, o):
    for rep in range(2):
        if rep == 1:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _lib.call("grace_topk_stream_probe", g.data_ptr(), r.data_ptr(), o.data_ptr(), n, 0, ws.data_ptr(), ws.numel(),
                  ops._stream())
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3


for rnd in range(1):
    for S in [0, 2, 4, 8, 16, 24, 32, 48, 64]:
        rs = [torch.empty(n, device=dev) for _ in range(4)]
        sp = torch.empty(S << 28, device=dev) if S else None   # S GiB
        outs = [torch.empty(n, device=dev) for _ in range(3)]
        us = [probe(r, o) for o in outs for r in rs]
        print(f"round {rnd} spacer {S:2d} GiB: pairs min {min(us):6.1f} max {max(us):6.1f} us; fast (< 178 us) "
              f"{sum(u < 178 for u in us)} of {len(us)}", flush=True)
        del rs, outs, sp
        torch.cuda.synchronize()
        torch.cuda.empty_cache()   # the next configuration allocates afresh (hipMalloc), not from torch's cache
