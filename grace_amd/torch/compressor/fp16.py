"""grace_dl/torch/compressor/fp16.py: identical to grace_dl/dist/compressor/fp16.py apart from the base-class
import, so the dist codec is the implementation (grace_amd/dist/compressor/fp16.py)."""
from grace_amd.dist.compressor.fp16 import FP16Compressor

__all__ = ["FP16Compressor"]
