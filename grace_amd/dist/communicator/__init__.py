"""Communicators mirroring grace_dl/dist/communicator/*.py over torch.distributed (RCCL on ROCm)."""
