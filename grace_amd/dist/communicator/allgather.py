"""Allgather communicator (grace_dl/dist/communicator/allgather.py:7-45) over torch.distributed
(RCCL on ROCm).

Differences from the reference that callers cannot observe:
  * each payload tensor moves with one ``all_gather_into_tensor`` into a contiguous rank-major
    buffer (no per-rank list of tensors), and compressors that provide
    ``decode_aggregate_gathered`` decode + aggregate + average all W payloads in one native pass;
  * at world_size 1 no collective is issued (the gathered list is the local payload), so no
    process group is required;
  * variable-size payloads exchange their sizes as a tensor on the payload's own device
    (the reference hard-codes ``.cuda()``, allgather.py:16).
"""
import torch
import torch.distributed as dist

from grace_amd.dist import Communicator
from grace_amd.dist._util import divide


def _gather_flat(t, world_size):
    flat = t.contiguous().view(-1)
    if world_size == 1:
        return flat
    out = torch.empty(world_size * flat.numel(), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat)
    return out


class Allgather(Communicator):
    def send_receive(self, tensors, name, ctx):
        W = int(self.world_size)
        if self.compressor.tensors_size_are_same:
            gathered = [_gather_flat(t, W) for t in tensors]
            fast = getattr(self.compressor, "decode_aggregate_gathered", None)
            if fast is not None:
                out = fast(gathered, ctx, W)
                if out is not None:
                    return out
            per_rank = [[g.view(W, -1)[r].view(t.shape) for g, t in zip(gathered, tensors)] for r in range(W)]
        else:
            gathered, sizes = self._gather_variable(tensors, W)
            fast = getattr(self.compressor, "decode_aggregate_variable", None)
            if fast is not None:
                out = fast(gathered, sizes, ctx, W)
                if out is not None:
                    return out
            per_rank = [[g.view(W, -1)[r][:sizes[r][j]] for j, g in enumerate(gathered)] for r in range(W)]
        decompressed_list = [self.compressor.decompress(tc, ctx) for tc in per_rank]
        tensors_aggregated = self.compressor.aggregate(decompressed_list)
        return divide(tensors_aggregated, W) if self.compressor.average else tensors_aggregated

    @staticmethod
    def _gather_variable(tensors, W):
        """Size exchange + padded all-gather (allgather.py:15-38).  Returns the rank-major padded
        buffers (one per payload tensor, W * max_size) and sizes[rank][tensor]."""
        if W == 1:
            return [t.contiguous().view(-1) for t in tensors], [[t.numel() for t in tensors]]
        dev = tensors[0].device
        local_sizes = torch.tensor([t.numel() for t in tensors], dtype=torch.int64, device=dev)
        all_sizes = torch.empty(W * len(tensors), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(all_sizes, local_sizes)
        sizes = all_sizes.view(W, len(tensors)).cpu().tolist()
        gathered = []
        for j, t in enumerate(tensors):
            max_size = max(sizes[r][j] for r in range(W))
            flat = t.contiguous().view(-1)
            if flat.numel() != max_size:
                padded = torch.zeros(max(max_size, 1), dtype=flat.dtype, device=flat.device)[:max_size]
                padded[:flat.numel()] = flat
                flat = padded
            out = torch.empty(W * max_size, dtype=flat.dtype, device=flat.device)
            if max_size:
                dist.all_gather_into_tensor(out, flat)
            gathered.append(out)
        return gathered, sizes
