"""Horovod-flavour API (grace_dl/torch/__init__.py:1-58) on torch.distributed (RCCL on ROCm).

The reference's ``grace_dl.torch`` drives Horovod's ``*_async`` collectives from autograd hooks:
``send_step`` (compensate -> compress -> update -> async_send) when a gradient is ready and
``receive_step`` (wait_receive -> decompress -> aggregate) before the optimizer step.  Here the
same split runs on ``torch.distributed`` work handles (``async_op=True``), which on RCCL are
stream-ordered: the collectives overlap the rest of the backward pass on the GPU.

``grace_amd.torch.compressor`` / ``.memory`` mirror ``grace_dl.torch.compressor`` / ``.memory``
module for module.  Six codecs compute something different from their dist copies (qsgd,
threshold, randomk, topk, powersgd, onebit's decode; DgcMemory's constructor) and have their own
implementations there; the others are the dist codecs, whose reference files differ only in the
base-class import.
"""
from abc import ABC, abstractmethod

from grace_amd.dist import Compressor, Memory  # noqa: F401  (same interfaces)


class Communicator(ABC):
    """async_send / wait_receive split of one gradient's exchange (grace_dl/torch/__init__.py:37-58)."""

    @abstractmethod
    def async_send(self, tensors, name):
        raise NotImplementedError("async_send was not implemented.")

    @abstractmethod
    def wait_receive(self, handles, ctx):
        raise NotImplementedError("wait_receive was not implemented.")

    def __init__(self, compressor, memory):
        self.compressor = compressor
        self.memory = memory

    def send_step(self, tensor, name):
        tensor = self.memory.compensate(tensor, name)
        tensors_compressed, ctx = self.compressor.compress(tensor, name)
        self.memory.update(tensor, name, self.compressor, tensors_compressed, ctx)
        handles = self.async_send(tensors_compressed, name)
        return handles, ctx

    def receive_step(self, handles, ctx):
        return self.wait_receive(handles, ctx)
