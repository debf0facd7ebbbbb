"""AllToAll: two-phase compressed allreduce (grace_dl/dist/communicator/all_to_all.py:13-124) for
the quantisers (QSGD / QSGD_CUDA, TernGrad, Natural / Natural_CUDA).

  phase 1  the payload is padded, cut into W chunks and exchanged with one all_to_all per tensor;
           rank r decodes the W copies of chunk r and sums them in rank order
  phase 2  rank r re-compresses its aggregated chunk; the chunks are all-gathered, decoded,
           concatenated, cut back to n and (if the compressor averages) divided by W.

Differences from the reference:
  * padding is zeros.  The reference pads with ``torch.empty`` (all_to_all.py:39,43,62,88): the
    garbage codes decode into the padded tail and, for TernGrad, enter the last chunk's scale in
    phase 2, so its results depend on uninitialised memory.  With zeros the padded tail is inert
    (QSGD: exactly its own zero-padding semantics);
  * payloads move with ``all_to_all_single`` / ``all_gather_into_tensor`` on flat buffers, and
    compressors that provide the native hooks decode + aggregate all W chunks in one launch;
  * at world_size 1 no collective is issued.
"""
import math

import torch
import torch.distributed as dist

from grace_amd.dist import Communicator
from grace_amd.dist._util import divide


def _kind(compressor):
    if getattr(compressor, "wire", "int8") not in ("int8", "u8"):
        raise NotImplementedError("AllToAll chunks the element-wise codes: use the default wire format")
    kind = getattr(compressor, "a2a_kind", None)
    if kind:
        return kind
    from grace_amd.dist.compressor.natural import NaturalCompressor
    from grace_amd.dist.compressor.qsgd import _QSGDBase
    from grace_amd.dist.compressor.terngrad import TernGradCompressor
    if isinstance(compressor, _QSGDBase):
        return "qsgd"
    if isinstance(compressor, TernGradCompressor):
        return "terngrad"
    if isinstance(compressor, NaturalCompressor):
        return "natural"
    raise NotImplementedError(compressor)


def _padded(t, size):
    flat = t.contiguous().view(-1)
    if flat.numel() == size:
        return flat
    out = torch.zeros(size, dtype=flat.dtype, device=flat.device)
    out[:flat.numel()] = flat
    return out


def _exchange(t, W):
    """all_to_all of W equal chunks of a flat tensor (chunk w goes to rank w)."""
    if W == 1:
        return t
    out = torch.empty_like(t)
    dist.all_to_all_single(out, t)
    return out


def _gather(t, W):
    flat = t.contiguous().view(-1)
    if W == 1:
        return flat
    out = torch.empty(W * flat.numel(), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat)
    return out


class AllToAll(Communicator):

    def send_receive(self, tensors, name, ctx):
        comp = self.compressor
        W = int(self.world_size)
        kind = _kind(comp)
        n = ctx.numel()
        unit = W * comp.bucket_size if kind == "qsgd" else W
        n_pad = math.ceil(n / unit) * unit
        chunk = n_pad // W
        chunk_shape = torch.Size([chunk])

        # ---- phase 1: exchange chunks, decode the W copies of ours, sum in rank order
        codes = _exchange(_padded(tensors[0], n_pad), W)
        if kind == "qsgd":
            nb = n_pad // comp.bucket_size
            norms = _exchange(_padded(tensors[1], nb), W)
            per_rank = [(codes[w * chunk:(w + 1) * chunk], norms[w * (nb // W):(w + 1) * (nb // W)])
                        for w in range(W)]
            gathered = (codes, norms)
        elif kind == "terngrad":
            scalars = _gather(tensors[1], W)
            per_rank = [(codes[w * chunk:(w + 1) * chunk], scalars[w:w + 1]) for w in range(W)]
            gathered = (codes, scalars)
        else:
            per_rank = [(codes[w * chunk:(w + 1) * chunk],) for w in range(W)]
            gathered = (codes,)
        fast = getattr(comp, "a2a_decode_sum", None)
        agg = fast(gathered, chunk, W) if fast is not None else None
        if agg is None:
            agg = comp.aggregate([comp.decompress(list(p), chunk_shape) for p in per_rank])

        # ---- phase 2: re-compress our aggregated chunk, all-gather, decode, concatenate
        payload2, ctx2 = comp.compress(agg, name)
        gathered2 = [_gather(t, W) for t in payload2]
        fast = getattr(comp, "a2a_decode_concat", None)
        full = fast(gathered2, chunk, W) if fast is not None else None
        if full is None:
            if kind == "qsgd":
                nbc = chunk // comp.bucket_size
                parts = [(gathered2[0][w * chunk:(w + 1) * chunk], gathered2[1][w * nbc:(w + 1) * nbc])
                         for w in range(W)]
            elif kind == "terngrad":
                parts = [(gathered2[0][w * chunk:(w + 1) * chunk], gathered2[1][w:w + 1]) for w in range(W)]
            else:
                parts = [(gathered2[0][w * chunk:(w + 1) * chunk],) for w in range(W)]
            full = torch.cat([comp.decompress(list(p), ctx2) for p in parts])
        out = full[:n].view(ctx)
        return divide(out, W) if comp.average else out
