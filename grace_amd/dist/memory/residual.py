"""Residual error feedback (grace_dl/dist/memory/residual.py:4-20) with device-resident
residual buffers keyed by name, like the reference's ``residuals`` dict."""
from grace_amd import ops
from grace_amd.dist import Memory


class ResidualMemory(Memory):
    def __init__(self, beta=1.0, gamma=1.0):
        self.residuals = {}
        self.beta = beta
        self.gamma = gamma

    def compensate(self, tensor, name):
        """t = beta * r + gamma * g; the first step returns the tensor itself (residual.py:10-14)."""
        if name in self.residuals:
            r = self.residuals[name]
            return ops.axpby(r, tensor, self.beta, self.gamma).view(tensor.shape)
        return tensor

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        """r = t - decompress(compress(t))  (residual.py:16-20)."""
        tensor_decompressed = compressor.decompress(tensor_compressed, ctx)
        self.residuals[name] = ops.sub(tensor, tensor_decompressed)

    def state_dict(self):
        """Residual buffers for checkpointing (the reference keeps them in a plain dict only)."""
        return {k: v.detach().clone() for k, v in self.residuals.items()}

    def load_state_dict(self, state):
        self.residuals = {k: v.clone() for k, v in state.items()}
