"""grace_dl/torch/memory/powersgd.py: identical to grace_dl/dist/memory/powersgd.py apart from the base-class
import, so the dist memory is the implementation (grace_amd/dist/memory/powersgd.py)."""
from grace_amd.dist.memory.powersgd import PowerSGDMemory

__all__ = ["PowerSGDMemory"]
