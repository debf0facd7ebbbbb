"""grace_dl/torch/compressor/signum.py: identical to grace_dl/dist/compressor/signum.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/signum.py)."""
from grace_amd.dist.compressor.signum import SignumCompressor

__all__ = ["SignumCompressor"]
