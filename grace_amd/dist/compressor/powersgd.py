"""PowerSGD rank-r compression (grace_dl/dist/compressor/powersgd.py:7-65) on f32 MFMA kernels
(grace_amd/csrc/powersgd.hip).

1-D tensors pass through uncompressed.  M = tensor.view(n0, -1); q is a fresh normal draw
orthogonalised by Gram-Schmidt, or q_memory[name] (un-orthogonalised) when use_memory; P = M q,
all_reduce, / world_size, orthogonalise; Q = M^T P, all_reduce, / world_size; payload [] and ctx
(P, Q, shape); decompress = P Q^T.  As in the reference the all-reduces happen inside compress.
``rng='device'`` draws q on the GPU; ``rng='torch_cpu'`` uses torch's CPU normal_ stream.
"""
import torch
import torch.distributed as dist

from grace_amd import ops
from grace_amd.dist import Compressor


def orthogonalize(matrix):
    """In-place modified Gram-Schmidt on the columns (powersgd.py:7-18)."""
    return ops.orthogonalize_(matrix)


class PowerSGDCompressor(Compressor):

    def __init__(self, rank=1, use_memory=False, world_size=1, rng="device", one_pass=True, check_sync=False):
        super().__init__()
        self.one_pass = one_pass   # world size 1, rank 4: P and Q from one read of M (psgd_w1_pass)
        # check_sync: wait for the one-pass kernels after every compress and raise PowerSGDWaitError
        # on THIS call (default: the next call raises, so the step itself never blocks the host)
        self.check_sync = check_sync
        self.world_size = world_size
        self.q_memory = {}
        self.rank = rank
        self.use_memory = use_memory
        self.rng = rng
        self._step = 0

    def _normal(self, m, r, device, name):
        self._step += 1
        if self.rng == "torch_cpu":
            return torch.empty(m, r).normal_().to(device)
        return ops.normal((m, r), ops.step_seed("powersgd-q", name, self._step), device)

    def compress(self, tensor, name):
        if tensor.dim() == 1:
            return [tensor], None
        shape = tensor.size()
        matrix = ops.dev_f32(tensor).view(shape[0], -1)
        n, m = matrix.size()
        r = min(n, m, self.rank)
        distributed = self.world_size > 1 or (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)
        if self.one_pass and not distributed and self.world_size == 1 and ops.powersgd_w1_ok(matrix, r):
            # world size 1: nothing is all-reduced between the contractions, so P = orth(M q) and
            # Q = M^T P come out of ONE pass over M (Q = (M^T M q) R^-1, f64 accumulation; see
            # powersgd.hip psgd_w1_pass).  q needs no orthogonalisation first, as below.
            if self.use_memory and name in self.q_memory:
                p, q = ops.powersgd_w1_compress(matrix, q=self.q_memory[name])
            elif self.rng == "torch_cpu":
                p, q = ops.powersgd_w1_compress(matrix, q=self._normal(m, r, matrix.device, name))
            else:
                self._step += 1
                p, q = ops.powersgd_w1_compress(matrix, seed=ops.step_seed("powersgd-q", name, self._step))
            if self.check_sync:
                ops.powersgd_w1_check()
            ctx = p, q, shape
            if self.use_memory:
                self.q_memory[name] = q
            return [], ctx
        if self.use_memory and name in self.q_memory:
            p = ops.powersgd_p(matrix, self.q_memory[name])
        elif self.rng == "torch_cpu":
            q = self._normal(m, r, matrix.device, name)
            orthogonalize(q)
            p = ops.powersgd_p(matrix, q)
        else:
            # device draw inside the contraction.  The fresh q is not orthogonalised first: with
            # q = q0 R^-1 (q0's own QR), orthogonalize(M q) = orthogonalize(M q0) because R^-1 is
            # upper triangular with a positive diagonal, so P after the orthogonalisation below is
            # the reference's (powersgd.py:40-49) up to rounding -- one launch and q's buffer saved
            self._step += 1
            p = ops.powersgd_p_draw(matrix, r, ops.step_seed("powersgd-q", name, self._step))
        if self.world_size > 1 or (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            dist.all_reduce(p)
        if self.world_size != 1:
            p = ops.div_scalar(p, self.world_size).view(n, r)
        orthogonalize(p)
        q = ops.powersgd_qt(matrix, p)
        if self.world_size > 1 or (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            dist.all_reduce(q)
        if self.world_size != 1:
            q = ops.div_scalar(q, self.world_size).view(m, r)
        ctx = p, q, shape
        if self.use_memory:
            self.q_memory[name] = q
        return [], ctx

    def decompress(self, tensors, ctx):
        if ctx is None:
            tensor, = tensors
            return tensor
        p, q, tensor_shape = ctx
        out, _ = ops.powersgd_outer(p, q)
        return out.view(tensor_shape)
