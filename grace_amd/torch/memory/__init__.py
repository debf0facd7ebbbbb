"""Horovod-flavour memories (grace_dl/torch/memory/*.py).  efsignsgd, none, powersgd and residual are
identical to the dist copies apart from the base-class import; DgcMemory takes no world_size and
averages the clipping norm over the ranks (grace_dl/torch/memory/dgc.py:8-18)."""
