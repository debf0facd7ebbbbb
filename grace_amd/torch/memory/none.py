"""grace_dl/torch/memory/none.py: identical to grace_dl/dist/memory/none.py apart from the base-class
import, so the dist memory is the implementation (grace_amd/dist/memory/none.py)."""
from grace_amd.dist.memory.none import NoneMemory

__all__ = ["NoneMemory"]
