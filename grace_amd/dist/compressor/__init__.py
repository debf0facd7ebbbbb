"""Codecs mirroring grace_dl/dist/compressor/*.py, computed by libgrace_hip.so."""
