"""Does a re-read of a MALL-sized buffer come from the 256 MB Infinity Cache?  Times torch's sum
(a pure streaming read) over buffers of 32 MB .. 1 GB, each read back to back 20 times, with HIP
events: a buffer that fits the MALL and is re-read should exceed the HBM rate the 1 GB buffer
shows.  usage: python tools/mall_probe.py"""
import json

import torch

dev = torch.device("cuda")
res = []
for mb in (32, 64, 102, 160, 256, 512, 1024):
    n = mb * (1 << 20) // 4
    x = torch.randn(n, device=dev)
    for _ in range(3):
        x.sum()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        x.sum()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    res.append({"MB": mb, "us_per_read": round(us, 2), "GBps": round(n * 4 / us / 1e3, 1)})
    del x
print(json.dumps(res))
