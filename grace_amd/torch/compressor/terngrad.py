"""grace_dl/torch/compressor/terngrad.py draws ``uniform_(0, scalar.item())`` where the dist copy draws
``uniform_(0, 1) * scalar`` (terngrad.py:19-20).  Both round the exact product u * scalar to f32 once,
so the codewords are identical; the torchflav golden fixtures (tests/test_gpu_torch_flavour.py) pin
the dist kernel against the torch reference.  Implementation: grace_amd/dist/compressor/terngrad.py."""
from grace_amd.dist.compressor.terngrad import TernGradCompressor

__all__ = ["TernGradCompressor"]
