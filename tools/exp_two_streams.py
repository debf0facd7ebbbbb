"""Cross-bucket overlap experiment for the headline step: the same
Allgather(TopK 1 %, ResidualMemory).step at world 1 on 256 MiB buckets, with bucket j's steps always
on stream j % S.  The engine's workspaces and reused outputs are keyed by stream (ops.workspace), so
two streams give two independent in-flight steps.  Modes: 0 = serial on torch's default stream; 1 = serial on one created stream; 2 = two streams,
free-running (the main passes of two buckets then overlap and contend for HBM); 4 = the same
with three streams; 3 = two streams,
and bucket i+1's step waits for bucket i's MAIN pass only (ops.MainEvent rides on that dispatch
packet), so exactly the latency-bound finalize(i) and bracket(i+1) run side by side.  Interleaved
rounds in one process, wall-clock ms per bucket step (median over rounds); per-name step order is
unchanged, and every mode is checked bit-exact against a serial run on the default stream.
usage: python tools/exp_two_streams.py [--buffers 4] [--steps 40] [--rounds 5]"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.dist.communicator.allgather import Allgather  # noqa: E402
from grace_amd.dist.compressor.topk import TopKCompressor  # noqa: E402
from grace_amd.dist.memory.residual import ResidualMemory  # noqa: E402
from grace_amd.ops import MainEvent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--numel", type=int, default=1 << 26)
ap.add_argument("--buffers", type=int, default=4)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--modes", default="0,1,2,3,4", help="modes, in the order each round runs them")
args = ap.parse_args()

dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev)
grads = []
for j in range(args.buffers):
    gen.manual_seed(j + 1)
    grads.append(torch.randn(args.numel, device=dev, generator=gen))
torch.cuda.synchronize()
streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
MODES = tuple(int(m) for m in args.modes.split(","))
comms = {s: Allgather(TopKCompressor(0.01), ResidualMemory(), 1) for s in MODES}
evs = [MainEvent(), MainEvent()]


def one(S, comm, i):
    j = i % args.buffers
    st = torch.cuda.default_stream(dev) if S == 0 else streams[j % {1: 1, 2: 2, 3: 2, 4: 3}[S]]
    with torch.cuda.stream(st):
        if S == 3:
            if i > 0:
                evs[(i - 1) % 2].wait(st)
            evs[i % 2].arm()
        return comm.step(grads[j], f"b{j}")


def run(S, steps):
    for i in range(steps):
        one(S, comms[S], i)


def check(S):
    """the last step's outputs of every bucket, against a serial re-run on the default stream"""
    ref = Allgather(TopKCompressor(0.01), ResidualMemory(), 1)
    for i in range(args.buffers * 3):
        j = i % args.buffers
        o = one(S, comms_chk[S], i)
        torch.cuda.synchronize()
        r = ref.step(grads[j], f"b{j}")
        torch.cuda.synchronize()
        if not torch.equal(o, r):
            return False
    return True


comms_chk = {s: Allgather(TopKCompressor(0.01), ResidualMemory(), 1) for s in MODES}
ok = {S: check(S) for S in MODES}
for S in MODES:
    run(S, 2 * args.buffers)
torch.cuda.synchronize()
res = {S: [] for S in MODES}
for rnd in range(args.rounds):
    for S in MODES:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(S, args.steps)
        torch.cuda.synchronize()
        res[S].append((time.perf_counter() - t0) / args.steps * 1e3)
for S in MODES:
    ms = statistics.median(res[S])
    print({"mode": {0: "serial, default stream", 1: "serial", 2: "2 streams", 3: "2 streams, wait on main", 4: "3 streams"}[S], "buffers": args.buffers, "ms_per_step": round(ms, 4),
           "GB_per_s": round(4 * args.numel / ms / 1e6, 1), "bit_exact_vs_serial": ok[S],
           "rounds": [round(x, 4) for x in res[S]]}, flush=True)
