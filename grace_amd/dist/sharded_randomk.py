"""Sharded random-k + residual memory: ONE bucket split over the ranks, stepped exactly as the
single-GPU ``Allgather(RandomKCompressor(ratio), ResidualMemory(), 1).step`` steps the whole bucket
(randomk.py:6-41, residual.py:10-20, allgather.py:40-45) -- SURVEY.md §8e row "random-k: all ranks
derive the same idx from seed h and keep their own range".

Per step on rank r (shard = the bucket's elements [lo, lo + m)):
1. the k GLOBAL indices, identical on every rank: h = sum(bytes(name)) + step counter, torch's
   global generator reseeded with h as the reference does, the draws from the device generator keyed
   by h (``rng="device"``, RandomKCompressor's default) or torch's CPU stream (``rng="torch_cpu"``);
2. ``grace_randomk_shard_step``: t = beta r + gamma g over the shard, r' = t with this rank's drawn
   positions t - t, and the payload vals with t where this rank holds the index and +0 elsewhere;
3. ``dense="shard"``: this rank's slice of the result (0 + t at its drawn positions) is written by
   the same step -- no collective at all; ``dense="replicated"``: ONE all-reduce (sum) of the k
   values -- every index has exactly one owner, so the sum is the whole bucket's payload -- and the
   decode of the whole bucket (``grace_randomk_decode``).
The residual of a name is kept per rank (its shard).  No host synchronisation in a step.
``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator.
"""
import torch
import torch.distributed as dist

from grace_amd import ops


class NativeRandomKKernels:
    def indices(self, h, n, k, rng, device):
        if rng == "torch_cpu":
            return torch.randint(n, [k]).to(device)
        return ops.randomk_indices(h, n, k, device)

    def shard_step(self, g, res, has, beta, gamma, lo, idx, out):
        return ops.randomk_shard_step(g, res, has, beta, gamma, lo, idx, out=out)

    def decode(self, vals, idx, n):
        return ops.randomk_decode(vals, idx, n)


class ShardedRandomK:
    """Random-k + residual over one bucket whose elements are sharded across `group`."""

    def __init__(self, compress_ratio, group=None, dense="replicated", rng="device", beta=1.0, gamma=1.0,
                 kernels=None):
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        if rng not in ("device", "torch_cpu"):
            raise ValueError("rng must be 'device' or 'torch_cpu'")
        self.compress_ratio = compress_ratio
        self.group = group
        self.dense = dense
        self.rng = rng
        self.beta, self.gamma = beta, gamma
        self.k_ops = kernels or NativeRandomKKernels()
        self.global_step = 0          # one counter per instance, as RandomKCompressor
        self.residuals = {}           # name -> this rank's residual shard

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    @staticmethod
    def partition(n, world):
        """Every rank's [start, end) of an n-element bucket: equal contiguous ranges (multiples of 4
        elements but the last)."""
        per = ((n + world - 1) // world + 3) // 4 * 4
        return [(min(r * per, n), min((r + 1) * per, n)) for r in range(world)]

    def step(self, shard, name, n):
        """This rank's shard (exactly partition(n, W)[rank]) of the n-element bucket `name` -> the
        step's result: the whole bucket (dense="replicated") or this rank's slice (dense="shard").
        The residual of `name` is updated in place."""
        K = self.k_ops
        world, rank = self._world()
        g = shard.reshape(-1)
        lo, hi = self.partition(int(n), world)[rank]
        if g.numel() != hi - lo:
            raise ValueError(f"ShardedRandomK: rank {rank} holds {g.numel()} elements, its range is {hi - lo}")
        h = sum(bytes(name, encoding="utf8"), self.global_step)
        self.global_step += 1
        torch.manual_seed(h)           # randomk.py:27 reseeds the global generator
        k = ops.ratio_k(int(n), self.compress_ratio)
        idx = K.indices(h, int(n), k, self.rng, g.device)
        res = self.residuals.get(name)
        has = res is not None and res.numel() == g.numel() and res.device == g.device
        if not has:
            res = torch.empty_like(g)
        out = torch.empty_like(g) if self.dense == "shard" else None
        if g.numel() == 0:
            vals = torch.zeros(k, dtype=torch.float32, device=g.device)
        else:
            vals = K.shard_step(g, res, has, self.beta, self.gamma, lo, idx, out)
        self.residuals[name] = res
        if self.dense == "shard":
            return out
        if world > 1:
            dist.all_reduce(vals, group=self.group)   # one owner per index: the sum is the payload
        return K.decode(vals, idx, int(n))
