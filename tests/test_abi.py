"""The C ABI library loads without a GPU and exports every symbol include/grace_hip.h declares
(no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    hdr = open(os.path.join(ROOT, "include", "grace_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(grace_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_functions():
    names = declared_functions()
    assert "grace_topk_residual_step" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    from grace_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"native library not built: {_lib.LIB_PATH}")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_table_matches_header():
    from grace_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_version_and_error_channel():
    from grace_amd import _lib
    lib = _lib.load()
    assert lib.grace_version() >= 100
    # an argument error is reported without touching the device
    st = lib.grace_axpby(None, None, 1.0, 1.0, None, 10, None)
    assert st == -1
    assert b"grace_axpby" in lib.grace_last_error()


def test_product_path_refuses_cpu_tensors():
    import torch
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.ops import GraceDeviceError
    with pytest.raises(GraceDeviceError):
        TopKCompressor(0.01).compress(torch.randn(100), "w")
