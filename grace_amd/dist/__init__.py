"""The three abstract roles of the GRACE API, same names and call contracts as
grace_dl/dist/__init__.py:4-51, so caller code is unchanged.

One addition, invisible to callers: ``Communicator.step`` asks the compressor for a fused native
plan (``fused_step``) and, when the (compressor, memory, communicator) triple supports one, runs
compensate -> compress -> update -> send_receive as one device pipeline.  The result is identical
to the four-call composition (tests/test_gpu_topk.py::test_topk_residual_golden_sequence runs
both paths against the reference's golden 3-step sequence; the QSGD / TernGrad / natural / fp16
fused steps have their own fused-equals-unfused tests in tests/test_gpu_quant.py).
"""
from abc import ABC, abstractmethod


class Memory(ABC):
    @abstractmethod
    def compensate(self, tensor, name):
        """Update the tensor with the residuals."""
        raise NotImplementedError("compensate was not implemented.")

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        """Update the residuals."""
        pass


class Compressor(ABC):
    """Interface for compressing and decompressing a given tensor."""

    def __init__(self, average=True, tensors_size_are_same=True):
        self.average = average
        self.tensors_size_are_same = tensors_size_are_same

    @abstractmethod
    def compress(self, tensor, name):
        """Compresses a tensor and returns it with the context needed to decompress it."""
        raise NotImplementedError("compress was not implemented.")

    @abstractmethod
    def decompress(self, tensors, ctx):
        """Decompress the tensor with the given context."""
        raise NotImplementedError("decompress was not implemented.")

    def aggregate(self, tensors):
        """Aggregate a list of tensors: Python ``sum`` in rank order, on the device."""
        from .. import ops
        if tensors and getattr(tensors[0], "is_cuda", False):
            return ops.sum_rank_order(tensors).view(tensors[0].shape)
        return sum(tensors)

    # optional fast path used by Communicator.step; returns None when not applicable
    def fused_step(self, communicator, tensor, name):
        return None


class Communicator(ABC):
    @abstractmethod
    def send_receive(self, tensors, name, ctx):
        raise NotImplementedError("send was not implemented.")

    def __init__(self, compressor, memory, world_size):
        self.compressor = compressor
        self.memory = memory
        self.world_size = world_size

    def step(self, tensor, name):
        fused = self.compressor.fused_step(self, tensor, name)
        if fused is not None:
            return fused
        tensor = self.memory.compensate(tensor, name)
        tensors_compressed, ctx = self.compressor.compress(tensor, name)
        self.memory.update(tensor, name, self.compressor, tensors_compressed, ctx)
        return self.send_receive(tensors_compressed, name, ctx)
