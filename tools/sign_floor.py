"""The floor of a 4 MiB streaming kernel: grace_sign_step_w1 (read 4 MiB f32, write 4 MiB f32) next
to the 2-read / 2-write probe moving the same 8 MiB (n = 512 Ki per array) and the encoder-mix probe,
each over 64 rotated buffer sets (past the 256 MB MALL) -- run under rocprofv3 --kernel-trace --stats
for the per-kernel durations.  With GAP > 0 a torch.cuda._sleep(GAP cycles) kernel precedes every
launch, so each one starts on an idle memory system as in the launch-bound bench step.
usage: python tools/sign_floor.py [reps] [gap]"""
import sys

import torch

from grace_amd import _lib, ops

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda")
nb = 64
n = 1 << 20
xs = [torch.randn(n, device=dev) for _ in range(nb)]
outs = [torch.empty(n, device=dev) for _ in range(nb)]
half = n // 2
pr = [tuple(torch.zeros(half, device=dev) for _ in range(3)) for _ in range(nb)]
st = ops._stream()
gap = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # cycles of torch.cuda._sleep before every launch


def space():
    if gap:
        torch.cuda._sleep(gap)


for i in range(reps):
    space()
    _lib.call("grace_sign_step_w1", xs[i % nb].data_ptr(), None, outs[i % nb].data_ptr(), n, st)
for v in (0, 3, 4):
    for i in range(reps):
        r, g, o = pr[i % nb]
        space()
        _lib.call("grace_hbm_probe", r.data_ptr(), g.data_ptr(), o.data_ptr(), half, v, st)
for v in (6, 8):
    for i in range(reps):
        space()
        _lib.call("grace_hbm_probe", xs[i % nb].data_ptr(), xs[i % nb].data_ptr(), outs[i % nb].data_ptr(), n, v, st)
torch.cuda.synchronize()
print("done")
