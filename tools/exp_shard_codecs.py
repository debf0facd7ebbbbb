"""Per-rank device time of the sharded §8e codecs at W = 8 without the collective (VERDICT r5
item 4): one process plays every rank of ShardedTernGrad, ShardedQuant("qsgd") and
ShardedPowerSGD with the collectives stubbed out (an all-reduce does nothing; an all-gather copies
the rank's own block into every slot with a torch copy kernel), so that what runs on the device is exactly one rank's kernels: the
encode into its send record and the decode of the whole bucket through the gathered records.
configs[2]'s 161 ResNet-50 tensors as one bucket (TernGrad, QSGD 127 / bucket 128) and configs[3]'s
4096 x 4096 matrix (PowerSGD rank 4).  Run under rocprofv3 --kernel-trace --stats: the grace
kernels' total time divided by the rank-steps printed here is the per-rank device time per step.
Also prints the event-timed wall time per rank-step (host submission included).
usage: python tools/exp_shard_codecs.py [W]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import resnet50_shapes  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
STEPS = 10
dev = torch.device("cuda", 0)


class StubDist:
    """torch.distributed as one rank of W sees it, with the data movement left out."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank

    def is_available(self):
        return True

    def is_initialized(self):
        return True

    def get_world_size(self, group=None):
        return self.world

    def get_rank(self, group=None):
        return self.rank

    def all_gather_into_tensor(self, out, inp, group=None):
        # every rank's block = this rank's (a torch copy, not a grace kernel: outside the per-rank
        # sum) -- so the decode reads real codes, norms, partials and factors
        out.view(self.world, -1).copy_(inp.reshape(1, -1).expand(self.world, -1))

    def all_reduce(self, t, op=None, group=None):
        pass


def run(label, make, inputs, step):
    """make(): a new engine; inputs[r]: rank r's shard; step(eng, x): one step"""
    import grace_amd.dist.sharded_powersgd as sp
    import grace_amd.dist.sharded_quant as sq
    import grace_amd.dist.sharded_terngrad as st
    engines = [make() for _ in range(W)]
    walls = []
    for s in range(STEPS + 2):
        for r in range(W):
            stub = StubDist(W, r)
            sq.dist = st.dist = sp.dist = stub
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            step(engines[r], inputs[r])
            b.record()
            if s >= 2:
                walls.append((a, b))
    torch.cuda.synchronize()
    w = statistics.median(x.elapsed_time(y) * 1e3 for x, y in walls)
    print(f"{label}: {STEPS * W} timed rank-steps (+ {2 * W} warm-up), event-timed wall per rank-step "
          f"{w:.1f} us (median)", flush=True)


def main():
    from grace_amd.dist.sharded_powersgd import ShardedPowerSGD
    from grace_amd.dist.sharded_quant import ShardedQuant
    from grace_amd.dist.sharded_terngrad import ShardedTernGrad
    sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
    n = sum(sizes)
    flat = torch.randn(n, device=dev) * 0.01
    tg = ShardedTernGrad(seed=7)
    parts = tg.partition(sizes, W)
    run("ShardedTernGrad (packed2 wire), ResNet-50 set", lambda: ShardedTernGrad(seed=7),
        [flat[a:b].clone() for a, b in parts], lambda e, x: e.step(x, sizes))
    qs = ShardedQuant("qsgd", quantum_num=127, bucket_size=128, seed=7)
    parts = qs.partition(sizes, W)
    run("ShardedQuant(qsgd 127, bucket 128), ResNet-50 set",
        lambda: ShardedQuant("qsgd", quantum_num=127, bucket_size=128, seed=7),
        [flat[a:b].clone() for a, b in parts], lambda e, x: e.step(x, sizes))
    M = torch.randn(4096, 4096, device=dev)
    rows = ShardedPowerSGD.partition(4096, W)
    run("ShardedPowerSGD rank 4, 4096 x 4096", lambda: ShardedPowerSGD(4),
        [M[a:b].clone() for a, b in rows], lambda e, x: e.step(x, "w", 4096))


if __name__ == "__main__":
    main()
