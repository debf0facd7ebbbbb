"""Per-rank device cost of the top-k Allgather step at world W > 1, without the collective: the
main pass without the dense output, the payload sort, and the rank-ordered decode of W payloads
(W copies of payloads from W different buckets stand in for the gathered ones).  Event-timed
stages, median over rounds, on the 256 MiB headline bucket."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = 64 * 1024 * 1024
k = ops.ratio_k(n, 0.01)
dev = torch.device("cuda", 0)
W = int(os.environ.get("W", "8"))
gs = [torch.randn(n, device=dev) for _ in range(3)]
rs = [0.1 * torch.randn(n, device=dev) for _ in range(3)]
# W distinct sorted payloads for the decode
pays = []
rz = torch.zeros(n, device=dev)
for w in range(W):
    gw = torch.randn(n, device=dev)
    buf, _, _ = ops.topk_residual_step(gw, rz, False, 1.0, 1.0, k, out=None)
    pays.append(ops.sort_payload(buf, k, n).clone())
gathered = torch.cat(pays)
del gw, rz


def ev():
    return torch.cuda.Event(enable_timing=True)


SWAP = os.environ.get("SWAP", "1") == "1"   # the r05 step into a second residual buffer
rs2 = [torch.empty_like(r) for r in rs] if SWAP else None
res = {"main_step": [], "sort": [], "decode": [], "total": []}
for rnd in range(12):
    j = rnd % 3
    e = [ev() for _ in range(4)]
    e[0].record()
    if SWAP:
        buf, _, _ = ops.topk_residual_step_swap(gs[j], rs[j], True, 1.0, 1.0, k, rs2[j])
        rs[j], rs2[j] = rs2[j], rs[j]
    else:
        buf, _, _ = ops.topk_residual_step(gs[j], rs[j], True, 1.0, 1.0, k, out=None)
    e[1].record()
    sb = ops.sort_payload(buf, k, n)
    e[2].record()
    out = ops.sparse_aggregate_sorted(gathered, k, W, n, float(W))
    e[3].record()
    torch.cuda.synchronize()
    if rnd >= 2:
        res["main_step"].append(e[0].elapsed_time(e[1]) * 1e3)
        res["sort"].append(e[1].elapsed_time(e[2]) * 1e3)
        res["decode"].append(e[2].elapsed_time(e[3]) * 1e3)
        res["total"].append(e[0].elapsed_time(e[3]) * 1e3)
print({"W": W, "swap": SWAP, **{kk: round(statistics.median(v), 1) for kk, v in res.items()}}, flush=True)
