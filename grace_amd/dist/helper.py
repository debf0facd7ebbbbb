"""grace_from_params (grace_dl/dist/helper.py:1-102): same keys, same defaults, same classes.

Differences: ``communicator='broadcast'`` works (the reference omits ``rank``, helper.py:95-97);
``kernel`` for top-k and the ``*_cuda`` codec names select the same native HIP codecs.

Extra keys (ignored by the reference's helper, so a params dict stays valid for both): for the
variable-size codecs ``threshold`` and ``dgc``, ``exchange`` ('counts' | 'capacity'),
``capacity_margin`` and ``overflow`` ('retry' | 'defer') pick the W > 1 payload exchange
(grace_amd/dist/compressor/threshold.py, dgc.py): 'capacity' moves one fixed-size record per rank
with no host read in the common step.
"""


def _exchange_kwargs(params, default_overflow):
    kw = {}
    if 'exchange' in params:
        kw['exchange'] = params['exchange']
    if 'capacity_margin' in params:
        kw['capacity_margin'] = params['capacity_margin']
    kw['overflow'] = params.get('overflow', default_overflow)
    return kw


def grace_from_params(params):
    comp = params.get('compressor', 'none')
    mem = params.get('memory', 'none')
    comm = params.get('communicator', 'allreduce')
    if comp == 'dgc':
        from grace_amd.dist.compressor.dgc import DgcCompressor
        compressor = DgcCompressor(params.get('compress_ratio', 0.3), **_exchange_kwargs(params, 'retry'))
    elif comp == 'efsignsgd':
        from grace_amd.dist.compressor.efsignsgd import EFSignSGDCompressor
        compressor = EFSignSGDCompressor(params.get('lr', 0.1))
    elif comp == 'fp16':
        from grace_amd.dist.compressor.fp16 import FP16Compressor
        compressor = FP16Compressor()
    elif comp == 'natural':
        from grace_amd.dist.compressor.natural import NaturalCompressor
        compressor = NaturalCompressor()
    elif comp == 'natural_cuda':
        from grace_amd.dist.compressor.natural import NaturalCompressor_CUDA
        compressor = NaturalCompressor_CUDA()
    elif comp == 'none':
        from grace_amd.dist.compressor.none import NoneCompressor
        compressor = NoneCompressor()
    elif comp == 'onebit':
        from grace_amd.dist.compressor.onebit import OneBitCompressor
        compressor = OneBitCompressor()
    elif comp == 'powersgd':
        from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
        compressor = PowerSGDCompressor()
    elif comp == 'qsgd':
        from grace_amd.dist.compressor.qsgd import QSGDCompressor
        compressor = QSGDCompressor(params.get('quantum_num', 127), params.get('bucket_size', 128))
    elif comp == 'qsgd_cuda':
        from grace_amd.dist.compressor.qsgd import QSGDCompressor_CUDA
        compressor = QSGDCompressor_CUDA(params.get('quantum_num', 127), params.get('bucket_size', 128))
    elif comp == 'randomk':
        from grace_amd.dist.compressor.randomk import RandomKCompressor
        compressor = RandomKCompressor(params.get('compress_ratio', 0.3))
    elif comp == 'signsgd':
        from grace_amd.dist.compressor.signsgd import SignSGDCompressor
        compressor = SignSGDCompressor()
    elif comp == 'signum':
        from grace_amd.dist.compressor.signum import SignumCompressor
        compressor = SignumCompressor(params.get('momentum', 0.9))
    elif comp == 'terngrad':
        from grace_amd.dist.compressor.terngrad import TernGradCompressor
        compressor = TernGradCompressor()
    elif comp == 'threshold':
        from grace_amd.dist.compressor.threshold import ThresholdCompressor
        compressor = ThresholdCompressor(params.get('threshold', 0.01), **_exchange_kwargs(params, 'retry'))
    elif comp == 'topk':
        from grace_amd.dist.compressor.topk import TopKCompressor
        compressor = TopKCompressor(params.get('compress_ratio', 0.3), params.get('kernel', 'torch'))
    else:
        raise NotImplementedError(comp)

    if mem == 'dgc':
        from grace_amd.dist.memory.dgc import DgcMemory
        memory = DgcMemory(params.get('momentum', 0.9), params.get('gradient_clipping', False),
                           params['world_size'])
    elif mem == 'none':
        from grace_amd.dist.memory.none import NoneMemory
        memory = NoneMemory()
    elif mem == 'powersgd':
        from grace_amd.dist.memory.powersgd import PowerSGDMemory
        memory = PowerSGDMemory(compressor.q_memory, params.get('compress_rank', 1))
    elif mem == 'residual':
        from grace_amd.dist.memory.residual import ResidualMemory
        memory = ResidualMemory()
    elif mem == 'efsignsgd':
        from grace_amd.dist.memory.efsignsgd import EFSignSGDMemory
        memory = EFSignSGDMemory(params.get('lr', 0.1))
    else:
        raise NotImplementedError(mem)

    if comm == 'allreduce':
        from grace_amd.dist.communicator.allreduce import Allreduce
        return Allreduce(compressor, memory, params['world_size'])
    elif comm == 'allgather':
        from grace_amd.dist.communicator.allgather import Allgather
        return Allgather(compressor, memory, params['world_size'])
    elif comm == 'broadcast':
        from grace_amd.dist.communicator.broadcast import Broadcast
        return Broadcast(compressor, memory, params['world_size'], params.get('rank'))
    elif comm == 'alltoall':
        from grace_amd.dist.communicator.all_to_all import AllToAll
        return AllToAll(compressor, memory, params['world_size'])
    else:
        raise NotImplementedError(comm)
