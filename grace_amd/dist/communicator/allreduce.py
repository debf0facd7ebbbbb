"""Allreduce communicator (grace_dl/dist/communicator/allreduce.py:6-13): in-place sum of each
payload tensor, divide by W when the compressor averages, then decompress.  Valid only for
payloads that are linear in the gradient (none, fp16, random-k, PowerSGD's empty payload)."""
import torch.distributed as dist

from grace_amd.dist import Communicator
from grace_amd.dist._util import divide


class Allreduce(Communicator):

    def send_receive(self, tensors, name, ctx):
        W = int(self.world_size)
        out = []
        for tensor_compressed in tensors:
            if W > 1:
                dist.all_reduce(tensor_compressed)
            if self.compressor.average:
                tensor_compressed = divide(tensor_compressed, W)
            out.append(tensor_compressed)
        return self.compressor.decompress(out, ctx)
