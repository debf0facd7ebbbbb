"""grace_dl/torch/memory/residual.py: identical to grace_dl/dist/memory/residual.py apart from the base-class
import, so the dist memory is the implementation (grace_amd/dist/memory/residual.py)."""
from grace_amd.dist.memory.residual import ResidualMemory

__all__ = ["ResidualMemory"]
