"""grace_dl/torch/compressor/signsgd.py: identical to grace_dl/dist/compressor/signsgd.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/signsgd.py)."""
from grace_amd.dist.compressor.signsgd import SignSGDCompressor

__all__ = ["SignSGDCompressor"]
