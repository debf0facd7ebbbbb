"""Host logic of the recycled world-1 top-k output (grace_amd/ops.py OutputRecycler), on CPU tensors:
a result comes back only when nothing outside the cache holds it or a view of it, it was not
modified in place, and the name, size, device and stream match.  (The device side -- clearing the
previous non-zeros and the sparse main pass -- is tests/test_gpu_topk_recycle.py.)"""
import pytest
import torch

from grace_amd import ops


@pytest.fixture(autouse=True)
def _cpu_stream(monkeypatch):
    state = {"s": 0}
    monkeypatch.setattr(ops, "_stream", lambda: state["s"])
    return state


def _step(rec, name, like):
    out, prev = rec.take(name, like)
    idx = torch.arange(4, dtype=torch.int32)
    rec.keep(name, out, idx)
    return out, prev


def test_dropped_result_comes_back_with_its_indices():
    rec = ops.OutputRecycler()
    like = torch.empty(100)
    out, prev = _step(rec, "b", like)
    assert prev is None and rec.misses == 1
    p = out.data_ptr()
    del out
    out, prev = _step(rec, "b", like)
    assert prev is not None and out.data_ptr() == p and rec.hits == 1
    assert torch.equal(prev, torch.arange(4, dtype=torch.int32))


def test_held_result_or_view_is_never_handed_back():
    rec = ops.OutputRecycler()
    like = torch.empty(100)
    held, _ = _step(rec, "b", like)
    out, prev = _step(rec, "b", like)
    assert prev is None and out.data_ptr() != held.data_ptr()
    view = out.view(10, 10)[2:]
    del out
    out2, prev = _step(rec, "b", like)
    assert prev is None and out2.data_ptr() != view.data_ptr()


def test_edited_result_is_not_handed_back():
    rec = ops.OutputRecycler()
    like = torch.empty(100)
    out, _ = _step(rec, "b", like)
    out.add_(1.0)                      # in place: the version counter moves
    p = out.data_ptr()
    del out
    out, prev = _step(rec, "b", like)
    assert prev is None and out.data_ptr() != p


def test_other_name_size_or_stream_allocates(_cpu_stream):
    rec = ops.OutputRecycler()
    out, _ = _step(rec, "a", torch.empty(100))
    del out
    _, prev = _step(rec, "b", torch.empty(100))        # another name
    assert prev is None
    _, prev = _step(rec, "a", torch.empty(101))        # another size
    assert prev is None
    out, _ = _step(rec, "c", torch.empty(100))
    del out
    _cpu_stream["s"] = 7                                 # another stream
    _, prev = _step(rec, "c", torch.empty(100))
    assert prev is None


def test_refcount_model_selftest_and_gate(monkeypatch):
    """the reuse checks rest on CPython / torch reference counts.  The import-time
    self-test replays their exact pattern and must accept this interpreter; with the gate off
    (as it would be on an interpreter that counts differently) nothing is ever handed back."""
    assert ops._refcount_selftest() and ops.REUSE_OK
    monkeypatch.setattr(ops, "REUSE_OK", False)
    rec = ops.OutputRecycler()
    like = torch.empty(100)
    out, _ = _step(rec, "b", like)
    del out
    out, prev = _step(rec, "b", like)
    assert prev is None and rec.hits == 0 and rec.misses == 2


def test_residual_spare_buffer_respects_holders():
    """ResidualMemory.spare_for (the world > 1 step's second residual buffer) reuses the name's
    previous residual only when nothing outside the memory holds it or a view of it."""
    from grace_amd.dist.memory.residual import ResidualMemory
    mem = ResidualMemory()
    like = torch.empty(64)
    a = mem.spare_for("w", like)
    mem.retire("w", a)
    pa = a.data_ptr()
    del a
    b = mem.spare_for("w", like)
    assert b.data_ptr() == pa                     # dropped: reused
    mem.retire("w", b)
    held = b                                      # the caller keeps its old residual
    del b
    c = mem.spare_for("w", like)
    assert c.data_ptr() != held.data_ptr()        # held: a fresh buffer
    mem.retire("w", c)
    v = c[3:]
    del c
    d = mem.spare_for("w", like)
    assert d.data_ptr() != v.data_ptr() - 12      # a view held: a fresh buffer
