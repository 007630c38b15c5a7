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
    assert lib.pcore_abi_version() == 7


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


def test_debug_covariances_rejects_k_outside_1_16():
    """pcore_debug_covariances validates 1 <= k <= 16 (pcore.h) before any launch."""
    lib = _native.load()
    lib.pcore_debug_covariances.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                                    ctypes.c_void_p]
    for k in (0, 17, -1):
        assert lib.pcore_debug_covariances(None, None, None, 0, k, None, None) == _native.PCORE_E_INVALID_ARG
