"""Threshold sparsification (grace_dl/dist/compressor/threshold.py:6-27): every element with
|x| >= min(threshold, max(x)) (signed max, as the reference), ascending index order, payload
[values f32[m], indices int32[m]] with m data-dependent (tensors_size_are_same=False).

Variable-size exchange.  The reference's step syncs the host twice: torch.where sizes the payload
(threshold.py:17) and Allgather exchanges the sizes as a CUDA tensor and reads them back
(allgather.py:15-18).  ``fused_step`` (Allgather with NoneMemory / ResidualMemory) needs ONE host
read: the count is finished on the device (recount decided there too), the W counts are
all-gathered on the device, and a single read of those W counts sizes both the local payload and
the padded exchange buffer -- the exchange itself adds no synchronisation."""
import numpy as np
import torch
import torch.distributed as dist

from grace_amd import _lib, ops
from grace_amd.dist import Compressor
from grace_amd.dist.communicator.allgather import Allgather
from grace_amd.dist.memory.none import NoneMemory
from grace_amd.dist.memory.residual import ResidualMemory


class ThresholdCompressor(Compressor):

    def __init__(self, threshold):
        super().__init__(tensors_size_are_same=False)
        self.threshold = threshold

    def compress(self, tensor, name):
        values, indices = ops.threshold_compress(tensor, self.threshold)
        return [values, indices], tensor.size()

    def decompress(self, tensor_compressed, ctx):
        values, indices = tensor_compressed
        return ops.sparse_decode(values, indices, ctx.numel()).view(ctx)

    def decode_aggregate_variable(self, gathered, sizes, ctx, world_size):
        """Variable-size Allgather: rank-ordered scatter-add of the W padded payloads."""
        vals, idx = gathered
        if not vals.is_cuda:
            return None
        stride = vals.numel() // world_size
        counts = [int(sizes[r][0]) for r in range(world_size)]
        out = ops.sparse_aggregate(vals, idx, stride, counts, world_size, ctx.numel(),
                                   world_size if self.average else 1)
        return out.view(ctx)

    def fused_step(self, communicator, tensor, name):
        mem = communicator.memory
        if not (communicator.__class__ is Allgather and type(mem) in (NoneMemory, ResidualMemory)
                and isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dtype == torch.float32):
            return None
        W = int(communicator.world_size)
        g = ops.dev_f32(tensor)
        n = g.numel()
        dev = g.device
        # compensate (residual.py:10-14): t = beta r + gamma g, computed straight into the buffer that
        # becomes the new residual; the first step's t is the tensor itself (copied for the residual)
        if type(mem) is ResidualMemory:
            r = mem.residuals.get(name)
            t = ops.axpby(r, g, mem.beta, mem.gamma) if r is not None and r.numel() == n else g.clone()
        else:
            t = g
        ws = ops.workspace("threshold", _lib.query("grace_threshold_workspace_bytes", n), dev)
        _lib.call("grace_threshold_count_dev", t.data_ptr(), n, float(np.float32(self.threshold)), ws.data_ptr(),
                  ops._stream())
        cnt = ws[4:8].view(torch.int32)
        if W > 1:
            counts_dev = torch.empty(W, dtype=torch.int32, device=dev)
            dist.all_gather_into_tensor(counts_dev, cnt)
        else:
            counts_dev = cnt
        counts = [int(c) for c in counts_dev.cpu().tolist()]     # the step's ONE host read
        m, cap = counts[dist.get_rank() if W > 1 else 0], max(max(counts), 1)
        send = torch.empty(2 * cap, dtype=torch.float32, device=dev)     # [vals | idx], padded to the max
        vals, idx = send[:m], send[cap:cap + m].view(torch.int32)
        if m:
            _lib.call("grace_threshold_write", t.data_ptr(), n, ws.data_ptr(), vals.data_ptr(), idx.data_ptr(),
                      ops._stream())
        if type(mem) is ResidualMemory:      # r = t - decompress(payload) (residual.py:16-20)
            _lib.call("grace_sparse_sub", vals.data_ptr(), idx.data_ptr(), m, t.data_ptr(), ops._stream())
            mem.residuals[name] = t.view(tensor.shape)
        if W > 1:
            recv = torch.empty(W * 2 * cap, dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(recv, send)
            out = ops.sparse_aggregate(recv, recv[cap:].view(torch.int32), 2 * cap, counts, W, n,
                                       W if self.average else 1)
        else:
            out = ops.sparse_aggregate(send, send[cap:].view(torch.int32), 0, counts, 1, n, 1)
        return out.view(tensor.shape)
