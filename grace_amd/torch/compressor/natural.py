"""grace_dl/torch/compressor/natural.py: the cupy NaturalCompressor of the dist flavour (the torch copy
has no _CUDA variant); implementation grace_amd/dist/compressor/natural.py."""
from grace_amd.dist.compressor.natural import NaturalCompressor

__all__ = ["NaturalCompressor"]
