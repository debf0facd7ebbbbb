"""grace_dl/torch/compressor/none.py: identical to grace_dl/dist/compressor/none.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/none.py)."""
from grace_amd.dist.compressor.none import NoneCompressor

__all__ = ["NoneCompressor"]
