"""Host logic of the segmented top-k (grace_amd/dist/segmented.py) on CPU: the memoised segment-list
normalisation must never hand back a stale result (an in-place edit of the same list, a tuple after
a list, numpy integers), and the per-segment tables it keys must follow the sizes.  (The device side
is tests/test_gpu_harness.py.)"""
import numpy as np
import pytest
import torch

from grace_amd import ops
from grace_amd.dist.segmented import SegmentedTopK


@pytest.fixture(autouse=True)
def _cpu_stream(monkeypatch):
    monkeypatch.setattr(ops, "_stream", lambda: 0)


def test_memo_sees_in_place_edits():
    e = SegmentedTopK(0.01)
    sizes = [10, 20000, 30]
    assert e._norm_sizes(sizes) == (20040, (10, 20000, 30))
    assert e._norm_sizes(sizes) == (20040, (10, 20000, 30))
    sizes[1] = 9000
    assert e._norm_sizes(sizes) == (9040, (10, 9000, 30))
    sizes.append(5)
    assert e._norm_sizes(sizes) == (9045, (10, 9000, 30, 5))


def test_memo_across_sequence_types():
    e = SegmentedTopK(0.01)
    assert e._norm_sizes([4, 5]) == (9, (4, 5))
    assert e._norm_sizes((4, 6)) == (10, (4, 6))
    assert e._norm_sizes(torch.Size([7, 8])) == (15, (7, 8))
    t, s = e._norm_sizes([np.int64(3), np.int32(4)])
    assert t == 7 and s == (3, 4) and all(type(v) is int for v in s)
    assert e._norm_sizes([np.int64(3), np.int32(5)]) == (8, (3, 5))


def test_tables_follow_the_sizes():
    e = SegmentedTopK(0.01)
    dev = torch.device("cpu")
    a = [100, 50000, 70000]
    _, ta = e._norm_sizes(a)
    T1 = e.tables(ta, dev, True, True)
    assert T1["n"] == sum(a) and T1["n_large"] == 2 and T1["n_small"] == 1
    assert e.tables(ta, dev, True, True) is T1                 # cached
    b = [100, 50000, 60000]
    T2 = e.tables(b, dev, True, True)                         # a plain list, not the memo's tuple
    assert T2 is not T1 and T2["n"] == sum(b)
    assert len(T2["args"]) == 14 and T2["args"][-1] == sum(b)
