"""grace_dl/torch/compressor/efsignsgd.py: identical to grace_dl/dist/compressor/efsignsgd.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/efsignsgd.py)."""
from grace_amd.dist.compressor.efsignsgd import EFSignSGDCompressor

__all__ = ["EFSignSGDCompressor"]
