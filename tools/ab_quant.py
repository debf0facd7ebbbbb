"""A/B the segmented QSGD(127, 128) encoder and the TernGrad compress (stats + encode) on the
ResNet-50 gradient set between builds of libgrace_hip, in ONE process on one device: interleaved
rounds over 3 rotated gradient sets (more than the MALL holds), per-build medians.
usage: python tools/ab_quant.py LIB_A LIB_B [...]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import resnet50_shapes  # noqa: E402
from grace_amd import ops  # noqa: E402

V, I64, I32, U64, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_float
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_qsgd_compress.argtypes = [V, V, V, I32, I64, I32, I32, I32, V, U64, V, V, V, V]
    L.grace_terngrad_compress.argtypes = [V, V, V, I32, I64, V, V, U64, V, V, V, V]
    L.grace_terngrad_workspace_bytes.restype = ctypes.c_size_t
    L.grace_terngrad_workspace_bytes.argtypes = [I64]
    L.grace_terngrad_unit.restype = I32
sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
n = sum(sizes)
dev = torch.device("cuda", 0)
xs = [torch.randn(n, device=dev) * 0.01 for _ in range(3)]
seg_off, bkt_off, nb = ops.seg_tables(sizes, 128, dev)
# unit tables per build (the TernGrad work-unit size is a build constant)
ttab = [ops.seg_tables(sizes, L.grace_terngrad_unit(), dev) for L in libs]
codes = torch.empty(n, dtype=torch.int8, device=dev)
norms = torch.empty(nb, device=dev)
scal = torch.empty(len(sizes), device=dev)
wss = [torch.zeros(L.grace_terngrad_workspace_bytes(ttab[i][2]), dtype=torch.uint8, device=dev)
       for i, L in enumerate(libs)]
stream = torch.cuda.current_stream().cuda_stream


def qsgd(L, i, j):
    L.grace_qsgd_compress(xs[j].data_ptr(), seg_off.data_ptr(), bkt_off.data_ptr(), len(sizes), nb, 127, 128, 0,
                          None, i, None, norms.data_ptr(), codes.data_ptr(), stream)


def tern(L, i, j):
    li = libs.index(L)
    tseg, tunit, nunits = ttab[li]
    L.grace_terngrad_compress(xs[j].data_ptr(), tseg.data_ptr(), tunit.data_ptr(), len(sizes), nunits, None, None,
                              i, codes.data_ptr(), scal.data_ptr(), wss[li].data_ptr(), stream)


res = {(w, i): [] for w in ("qsgd", "tern") for i in range(len(libs))}
for rnd in range(7):
    for w, fn in (("qsgd", qsgd), ("tern", tern)):
        for i, L in enumerate(libs):
            for s in range(3):
                fn(L, s, s % 3)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(30):
                fn(L, s, s % 3)
            e1.record()
            torch.cuda.synchronize()
            if rnd > 0:
                res[(w, i)].append(e0.elapsed_time(e1) / 30 * 1e3)
for i, p in enumerate(sys.argv[1:]):
    print({"lib": os.path.basename(p), "qsgd_compress_us": round(statistics.median(res[("qsgd", i)]), 2),
           "terngrad_compress_us": round(statistics.median(res[("tern", i)]), 2)})
