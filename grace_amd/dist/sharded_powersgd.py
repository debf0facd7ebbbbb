"""Sharded PowerSGD: ONE matrix M (n x m) split by rows over the ranks and compressed as the
single-GPU ``PowerSGDCompressor(rank)`` compresses it whole (powersgd.py:30-65, world 1: nothing to
average) -- SURVEY.md §8e row "PowerSGD: row-shard G.  P_shard = G_shard Q is local;
orthogonalisation needs the column dots; Q = Σ G_shardᵀ P_shard is an allreduce of f32[m x r]".

Per step on rank i (rows [lo, hi) of M):
1. P_i = M_i q with q the step's normal draws (identical on every rank: the device generator keyed
   by the step seed, drawn inside the contraction as the single-GPU compressor does);
2. ONE all-gather of the P_i blocks (n x r f32: 64 KiB at 4096 x 4), then every rank orthogonalises
   the whole P itself (Cholesky-QR in f64, grace_orthogonalize) -- identical on every rank, and the
   same input the single-GPU compressor orthogonalises, row for row;
3. Q_i = M_iᵀ P_i (rows [lo, hi) of P), ONE all-reduce (sum) of the m x r partials: Q = Mᵀ P;
4. decode: ``dense="replicated"`` every rank forms the whole P Qᵀ (it has both factors, no third
   collective); ``dense="shard"`` only its rows P_i Qᵀ.
Optional error feedback (``memory=True``, PowerSGDMemory, memory/powersgd.py:6-37): each rank keeps
its rows of the residual, t = M_i + r_i before the step and r_i = t - P_i Qᵀ after it (one pass).
The Q sum's order differs from the single-GPU contraction's, so results agree within f32 tolerance
(as PowerSGD's own parity is stated), not bit for bit.  No host synchronisation in a step.
``kernels`` defaults to the native HIP set; the CPU tests inject an oracle-backed emulator.
"""
import torch
import torch.distributed as dist

from grace_amd import ops


class NativePowerSGDKernels:
    """The HIP calls behind each step (GPU tensors only)."""

    def p_draw(self, M, r, seed, out=None):
        ops.dev_f32(M, "rows")   # a GPU f32 tensor, or GraceDeviceError
        return ops.powersgd_p_draw(M, r, seed, out=out)

    def orthogonalize_(self, P):
        return ops.orthogonalize_(P)

    def qt(self, M, P):
        ops.dev_f32(M, "rows")
        return ops.powersgd_qt(M, P)

    def outer(self, P, Q, M=None):
        """-> P Qᵀ, or with M the residual M - P Qᵀ"""
        out, res = ops.powersgd_outer(P, Q, M2d=M, want_out=M is None, want_residual=M is not None)
        return out if M is None else res

    def add(self, a, b):
        return ops.axpby(a.reshape(-1), b.reshape(-1), 1.0, 1.0).view(b.shape)


class ShardedPowerSGD:
    """Rank-r PowerSGD of one matrix whose rows are sharded across `group`."""

    def __init__(self, rank=4, group=None, dense="replicated", memory=False, kernels=None):
        if dense not in ("replicated", "shard"):
            raise ValueError("dense must be 'replicated' or 'shard'")
        self.rank = int(rank)
        self.group = group
        self.dense = dense
        self.memory = memory
        self.residuals = {}     # name -> this rank's rows of the residual
        self._steps = {}
        self.k_ops = kernels or NativePowerSGDKernels()

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    @staticmethod
    def partition(n_rows, world):
        """Every rank's [lo, hi) rows: equal contiguous blocks."""
        per = (n_rows + world - 1) // world
        return [(min(r * per, n_rows), min((r + 1) * per, n_rows)) for r in range(world)]

    def step(self, rows, name, n_rows):
        """This rank's rows (exactly partition(n_rows, W)[rank] of the n_rows x m matrix `name`) ->
        P Qᵀ (dense="replicated": n_rows x m) or this rank's rows of it (dense="shard")."""
        world, rank = self._world()
        K = self.k_ops
        if rows.dim() != 2:
            raise ValueError("ShardedPowerSGD: a rank's rows are a 2-D (rows x m) tensor")
        Mi = rows.contiguous() if rows.dtype == torch.float32 else rows.float().contiguous()
        lo, hi = self.partition(int(n_rows), world)[rank]
        if Mi.shape[0] != hi - lo:
            raise ValueError(f"ShardedPowerSGD: rank {rank} holds {Mi.shape[0]} rows, its block is {hi - lo}")
        m = Mi.shape[1]
        r = min(int(n_rows), m, self.rank)
        dev = Mi.device
        step = self._steps.get(name, 0) + 1
        self._steps[name] = step
        if self.memory:
            res = self.residuals.get(name)
            if res is not None and res.shape == Mi.shape:
                # t = M + r (memory/powersgd.py:16-25: tensor += residual), into a fresh buffer
                Mi = K.add(res, Mi)
        seed = ops.step_seed("powersgd-q", name, step)
        # the whole P on every rank: one all-gather of the row blocks.  Every block is `per` rows
        # except the last non-empty one, so the first n_rows gathered rows ARE P: P_i is drawn
        # straight into this rank's send block and nothing is copied back (the padding rows after
        # the last block are never read)
        per = max(b - a for a, b in self.partition(int(n_rows), world))
        if world > 1:
            send = torch.empty(per, r, dtype=torch.float32, device=dev)
            if hi > lo:
                K.p_draw(Mi, r, seed, out=send[:hi - lo])
            gathered = torch.empty(world * per, r, dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(gathered, send, group=self.group)
            P = gathered[:int(n_rows)]
        else:
            P = K.p_draw(Mi, r, seed) if hi > lo else torch.empty(0, r, dtype=torch.float32, device=dev)
        K.orthogonalize_(P)
        Pi = P[lo:hi]
        Q = K.qt(Mi, Pi) if hi > lo else torch.zeros(m, r, dtype=torch.float32, device=dev)
        if world > 1:
            dist.all_reduce(Q, group=self.group)
        if self.memory and hi > lo:
            self.residuals[name] = K.outer(Pi, Q, M=Mi)
        if self.dense == "shard":
            if hi == lo:
                return torch.empty(0, m, dtype=torch.float32, device=dev)
            return K.outer(Pi, Q)
        return K.outer(P, Q)
