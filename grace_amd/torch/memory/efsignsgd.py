"""grace_dl/torch/memory/efsignsgd.py: identical to grace_dl/dist/memory/efsignsgd.py apart from the base-class
import, so the dist memory is the implementation (grace_amd/dist/memory/efsignsgd.py)."""
from grace_amd.dist.memory.efsignsgd import EFSignSGDMemory

__all__ = ["EFSignSGDMemory"]
