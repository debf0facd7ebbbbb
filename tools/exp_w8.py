"""Single-GPU estimate of the DP-replica step's local work at world W (no collective): the
RES-mode top-k step (no dense output) + payload sort + the rank-ordered decode/aggregate of W
payloads (old: W scatters; new: index-sorted one-pass aggregate)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402


def timeit(fn, reps=10):
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


n = 64 * 1024 * 1024
k = n // 100
g = [torch.randn(n, device="cuda") for _ in range(3)]
r = [0.1 * torch.randn(n, device="cuda") for _ in range(3)]
it = iter(range(10 ** 9))
t_res = timeit(lambda: ops.topk_residual_step(g[next(it) % 3], r[next(it) % 3], True, 1.0, 1.0, k))
buf0 = ops.topk_compress(g[0], k)[0]
t_sort = timeit(lambda: ops.sort_payload(buf0, k, n))
for W in (2, 4, 8):
    bufs = [ops.topk_compress(g[w % 3] * (1 + w), k)[0] for w in range(W)]
    payload = torch.cat(bufs)
    sorted_payload = torch.cat([ops.sort_payload(b, k, n) for b in bufs])
    t_old = timeit(lambda: ops.sparse_aggregate(payload, payload[k:].view(torch.int32), 2 * k, [k] * W, W, n, W))
    t_new = timeit(lambda: ops.sparse_aggregate_sorted(sorted_payload, k, W, n, W))
    a = ops.sparse_aggregate(payload, payload[k:].view(torch.int32), 2 * k, [k] * W, W, n, W)
    b = ops.sparse_aggregate_sorted(sorted_payload, k, W, n, W)
    same = torch.equal(a.view(torch.int32), b.view(torch.int32))
    print(f"W={W}: res_step={t_res:.1f}us sort={t_sort:.1f}us agg_scatter={t_old:.1f}us agg_sorted={t_new:.1f}us "
          f"bit_equal={same}", flush=True)
