"""Small host helpers shared by the dist codecs."""
import torch

from .. import ops


def divide(t, world_size):
    """``t / world_size`` (allgather.py:45, allreduce.py:12).  Device tensors divide in the HIP
    library; host tensors can only come from foreign (non-grace_amd) compressors."""
    if t.is_cuda:
        return ops.div_scalar(t, world_size).view(t.shape)
    return t / world_size


def is_world1(communicator):
    return int(communicator.world_size) == 1


def same_dtype_device(a, b):
    return a.dtype == b.dtype and a.device == b.device


__all__ = ["divide", "is_world1", "same_dtype_device", "torch"]
