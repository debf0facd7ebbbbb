"""Diagnostic: psgd_w1_pass phase stamps (GRACE_STAMPS build) and per-kernel event times of the
world-1 PowerSGD compress on a 4096 x 4096 matrix.  Run on the GPU box:
    GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so python tools/exp_w1.py"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd import ops  # noqa: E402

n = m = int(os.environ.get("N", "4096"))
dev = torch.device("cuda", 0)
Ms = [torch.randn(n, m, device=dev) for _ in range(5)]
rows = []
for it in range(12):
    ws = ops.workspace("powersgd_w1", ops._lib.query("grace_powersgd_w1_workspace_bytes", n, m), dev)
    dbg = ws[256 + 2 * 4 * 16384: 256 + 2 * 4 * 16384 + 16384].view(torch.int64)
    dbg.zero_()
    dbg[6] = 2 ** 62
    dbg[1810] = 2 ** 62
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.powersgd_w1_compress(Ms[it % 5], seed=it)
    e1.record()
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().astype(np.int64)
    us = lambda a, b: (d[b] - d[a]) / 100.0
    nwg = 256
    wg = d[8: 8 + 4 * nwg].reshape(nwg, 4)
    t0 = d[6]
    ld = (wg[:, 0] - t0) / 100.0
    ex = (wg[:, 1] - wg[:, 0]) / 100.0
    en = (wg[:, 3] - t0) / 100.0
    f = d[1800:1812]
    fin = {"fin_prefetch": (f[1] - f[0]) / 100, "fin_gram": (f[2] - f[1]) / 100, "fin_chol": (f[3] - f[2]) / 100,
           "fin_solve": (f[4] - f[3]) / 100, "fin_wg0": (f[4] - f[0]) / 100, "fin_span": (f[11] - f[10]) / 100,
           "gap_pass_fin": (f[10] - d[7]) / 100}
    stt = (d[1200:1200 + nwg] - t0) / 100.0   # per-workgroup start
    rows.append({**fin, "start_med": float(np.median(stt)), "start_max": stt.max(),
                 "load_dur_med": float(np.median(ld - stt)), "load_dur_max": (ld - stt).max(), "ld_min": ld.min(), "ld_med": float(np.median(ld)), "ld_max": ld.max(),
                 "wait_med": float(np.median(ex)), "wait_max": ex.max(), "end_min": en.min(), "end_max": en.max(),"to_pphase_done": us(0, 1), "exchange_wait": us(1, 2), "to_qraw": us(2, 3), "qraw_to_end": us(3, 4),
                 "wg00_total": us(0, 4), "grid_span": (d[7] - d[6]) / 100.0, "two_kernels_event": e0.elapsed_time(e1) * 1e3})
print({k: round(statistics.median(r[k] for r in rows[2:]), 2) for k in rows[0]})
