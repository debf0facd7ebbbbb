"""grace_amd — MI355X-native gradient-compression codec engine.

Drop-in for sands-lab/grace's ``grace_dl.dist`` API (Compressor / Memory / Communicator and
``grace_from_params``), with every codec implemented as hand-written HIP kernels for gfx950 in
``libgrace_hip.so`` (C ABI: include/grace_hip.h).  Swap ``grace_dl.dist`` for ``grace_amd.dist``.
"""
__version__ = "0.1.0"
