"""Diagnostic: the bench's ddp_segmented step (ResNet-50 shapes, world 1) run 40 times for a
rocprofv3 kernel trace, under whichever library GRACE_HIP_LIB names (A/B and timing-only builds,
e.g. libgrace_hip_segnosmall.so whose prep leaves the small segments out)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from grace_amd.dist.segmented import SegmentedTopK  # noqa: E402
from grace_amd.harness import GradBucket, ShapeModel, step_segmented  # noqa: E402

dev = torch.device("cuda", 0)
bucket = GradBucket(ShapeModel(bench.resnet50_shapes(), dev))
bucket.flat.normal_()
eng = SegmentedTopK(0.01)
for _ in range(40):
    step_segmented(bucket, eng)
torch.cuda.synchronize()
print("done", os.environ.get("GRACE_HIP_LIB", "default"))
