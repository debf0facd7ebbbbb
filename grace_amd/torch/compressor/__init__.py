"""Horovod-flavour compressors (grace_dl/torch/compressor/*.py) on the HIP codec library.

Where the reference's torch copy computes something different from its dist copy, the class here
is its own implementation: qsgd (one global norm), threshold (strict >, int64 indices), randomk
(randperm: no replacement), topk (int64 indices, (numel, shape) ctx), powersgd (q from the memory,
averaged all-reduces), onebit (fixed decode).  The rest are the dist codecs: the reference's torch
files for them differ from the dist ones only in the base-class import (checked file by file with
diff; terngrad's uniform_(0, scalar) draw is pinned equal to uniform_(0, 1) * scalar by the
torchflav golden fixtures).
"""
