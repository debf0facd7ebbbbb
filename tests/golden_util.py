"""Loader for the committed golden fixtures (tests/golden/*.npz + manifest.json).

The fixtures were produced by tests/golden/gen_golden.py from the reference
implementation; this module only reads data (numpy.load, allow_pickle=False).
"""
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Case(dict):
    """Arrays of one fixture case plus its ``meta`` dict."""

    def __init__(self, meta, arrays):
        super().__init__(arrays)
        self.meta = meta
        self.name = meta["case"]


class Golden:
    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
            self.manifest = json.load(f)
        self._files = {}

    def _npz(self, family):
        if family not in self._files:
            with np.load(os.path.join(GOLDEN_DIR, family + ".npz"), allow_pickle=False) as z:
                self._files[family] = {k: z[k] for k in z.files}
        return self._files[family]

    def cases(self, family, codec=None, prefix=None):
        arrs = self._npz(family)
        out = []
        for meta in self.manifest[family]:
            if codec is not None and meta.get("codec") != codec:
                continue
            if prefix is not None and not meta["case"].startswith(prefix):
                continue
            pre = meta["case"] + "__"
            out.append(Case(meta, {k[len(pre):]: v for k, v in arrs.items() if k.startswith(pre)}))
        return out

    def case(self, family, name):
        for c in self.cases(family):
            if c.name == name:
                return c
        raise KeyError(name)


def same_bits(a, b):
    """Bitwise equality of two float arrays (NaN == NaN, +0 != -0)."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    return bool(np.array_equal(a.view(np.uint8), b.view(np.uint8)))


def topk_sets_match(x, idx_a, idx_b, k):
    """Index sets agree for |x| above the k-th key; tie counts at the k-th key agree."""
    from oracle.grace_oracle import abs_key
    key = abs_key(np.asarray(x).ravel())
    ia = np.sort(np.asarray(idx_a, dtype=np.int64))
    ib = np.sort(np.asarray(idx_b, dtype=np.int64))
    if ia.size != k or ib.size != k:
        return False
    kth = min(key[ia].min(), key[ib].min()) if k else 0
    if key[ia].min() != key[ib].min():
        return False
    above_a = ia[key[ia] > kth]
    above_b = ib[key[ib] > kth]
    return bool(np.array_equal(above_a, above_b)) and (ia.size - above_a.size == ib.size - above_b.size)
