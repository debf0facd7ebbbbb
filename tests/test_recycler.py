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
