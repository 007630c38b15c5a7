"""The C-ABI library loads and exports every symbol include/pcore.h declares (no compute calls)."""
import ctypes
import os
import re

from perception_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pcore.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcore_[a-z_]+)\s*\(", src)))


def test_header_declares_the_expected_entry_points():
    assert _declared() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    for name in _declared():
        assert hasattr(lib, name), name
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr)
    assert lib.pcore_abi_version() == 6


def test_library_is_gfx950_code():
    with open(_native.library_path(), "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_create_without_gpu_fails_cleanly():
    import torch

    if torch.cuda.is_available():
        return
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.pcore_create(0, ctypes.byref(h)) != 0
    assert lib.pcore_destroy(None) is None
