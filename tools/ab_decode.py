"""A/B the segmented decoders on the ResNet-50 gradient set (TernGrad decompress, QSGD(127, 128)
decompress, and sharded TernGrad's decode through 8 packed records) between builds of libgrace_hip,
in ONE process: interleaved rounds, 3 rotated code sets, per-build medians of 20 back-to-back
decodes, and a cross-build bit-exactness check of every output.
usage: python tools/ab_decode.py LIB_A LIB_B [...]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import resnet50_shapes  # noqa: E402
from grace_amd import ops  # noqa: E402

V, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
for L in libs:
    L.grace_terngrad_decompress.argtypes = [V, V, I64, I64, I32, V, I32, I64, I32, F, V, V]
    L.grace_qsgd_decompress.argtypes = [V, V, I64, I64, I32, V, V, I32, I64, I32, I32, I32, I32, F, V, V]
    L.grace_terngrad_decompress_records.argtypes = [V, I64, I32, V, I32, V, V, I32, I64, V, V]
sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
n = sum(sizes)
dev = torch.device("cuda", 0)
W = 8
codes = [torch.randint(-1, 2, (n,), dtype=torch.int8, device=dev) for _ in range(3)]
qcodes = [torch.randint(-127, 128, (n,), dtype=torch.int8, device=dev) for _ in range(3)]
scal = torch.rand(len(sizes), device=dev)
seg_off, bkt_off, nb = ops.seg_tables(sizes, 128, dev)
norms = torch.rand(nb, device=dev)
out = torch.empty(n, device=dev)
# 8 packed records of an even unit split (the sharded engine's layout)
unit = 16384
starts = []
a = 0
for s in sizes:
    starts += [a + j * unit for j in range((s + unit - 1) // unit)]
    a += s
U = (len(starts) + W - 1) // W
lo = [starts[min(r * U, len(starts) - 1)] if r * U < len(starts) else n for r in range(W)] + [n]
maxlen = max(lo[r + 1] - lo[r] for r in range(W))
pb = ((maxlen + (4 - maxlen % 4)) // 4 + 15) // 16 * 16
recs = [torch.randint(0, 256, (W * pb,), dtype=torch.uint8, device=dev) for _ in range(3)]
rank_lo = torch.tensor(lo, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def tern(L, j):
    L.grace_terngrad_decompress(codes[j].data_ptr(), scal.data_ptr(), n, len(sizes), 1, seg_off.data_ptr(),
                                len(sizes), n, 0, 1.0, out.data_ptr(), stream)


def qsgd(L, j):
    L.grace_qsgd_decompress(qcodes[j].data_ptr(), norms.data_ptr(), n, nb, 1, seg_off.data_ptr(), bkt_off.data_ptr(),
                            len(sizes), n, 127, 128, 0, 0, 1.0, out.data_ptr(), stream)


def trec(L, j):
    L.grace_terngrad_decompress_records(recs[j].data_ptr(), pb, W, rank_lo.data_ptr(), 1, scal.data_ptr(),
                                        seg_off.data_ptr(), len(sizes), n, out.data_ptr(), stream)


cases = {"tern_decode": tern, "qsgd_decode": qsgd, "tern_records_decode": trec}
ref = {}
for c, fn in cases.items():
    for i, L in enumerate(libs):
        fn(L, 0)
        torch.cuda.synchronize()
        o = out.clone()
        if i == 0:
            ref[c] = o
        elif not torch.equal(o.view(torch.int32), ref[c].view(torch.int32)):
            print(f"{c}: {sys.argv[1 + i]} differs from {sys.argv[1]}", flush=True)
res = {(c, i): [] for c in cases for i in range(len(libs))}
for rnd in range(8):
    for c, fn in cases.items():
        for i, L in enumerate(libs):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(20):
                fn(L, s % 3)
            e1.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                res[(c, i)].append(e0.elapsed_time(e1) / 20 * 1e3)
for c in cases:
    for i in range(len(libs)):
        print(f"{c:20s} {sys.argv[1 + i].rsplit('/', 1)[-1]:32s} {statistics.median(res[(c, i)]):7.2f} us", flush=True)
