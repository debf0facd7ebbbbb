"""grace_dl/torch/compressor/dgc.py: identical to grace_dl/dist/compressor/dgc.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/dgc.py)."""
from grace_amd.dist.compressor.dgc import DgcCompressor

__all__ = ["DgcCompressor"]
