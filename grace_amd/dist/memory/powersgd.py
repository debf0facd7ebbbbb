"""PowerSGD error feedback (grace_dl/dist/memory/powersgd.py:6-37): compensate adds the residual
IN PLACE (t += r) once the name has a q_memory entry, and draws a fresh normal q into the shared
q_memory; update stores r = t - P Q^T with the decompression fused into the same pass."""
from grace_amd import ops
from grace_amd.dist import Memory


class PowerSGDMemory(Memory):
    def __init__(self, q_memory, compress_rank=1, rng="device"):
        self.compress_rank = compress_rank
        self.q_memory = q_memory
        self.residuals = {}
        self.rng = rng
        self._step = 0

    def compensate(self, tensor, name):
        if tensor.dim() == 1:
            return tensor
        if name in self.q_memory:
            # tensor += residual, in place on any layout (a non-contiguous tensor is compensated
            # through a contiguous copy that is written back)
            flat = ops.dev_f32(tensor)
            ops.axpby(self.residuals[name], flat, 1.0, 1.0, out=flat)
            if not tensor.is_contiguous():
                tensor.copy_(flat.view(tensor.shape))
        shape = tensor.size()
        n = shape[0]
        m = 1
        for dim in shape[1:]:
            m = m * dim
        r = min(n, m, self.compress_rank)
        self._step += 1
        if self.rng == "torch_cpu":
            import torch
            self.q_memory[name] = torch.empty(m, r).normal_().to(tensor.device)
        else:
            self.q_memory[name] = ops.normal((m, r), ops.step_seed("powersgd-mem", name, self._step), tensor.device)
        return tensor

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        if ctx is None:
            return
        p, q, shape = ctx
        matrix = ops.dev_f32(tensor).view(shape[0], -1)
        _, res = ops.powersgd_outer(p, q, matrix, want_out=False, want_residual=True)
        self.residuals[name] = res.view(shape)
