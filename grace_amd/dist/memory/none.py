from grace_amd.dist import Memory


class NoneMemory(Memory):
    """No error feedback (grace_dl/dist/memory/none.py:4-11)."""

    def compensate(self, tensor, name):
        return tensor

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        pass
