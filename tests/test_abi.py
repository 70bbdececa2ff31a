"""C ABI checks that need no GPU: the library builds, loads, and exports every symbol
declared in include/frei_hip.h with the ctypes signatures the host layer binds."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "frei_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(frei_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    for must in ("frei_sweep", "frei_run", "frei_kappa", "frei_propagate_fluxes",
                 "frei_set_table", "frei_comm_init"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from frei_amd import _native as N
    lib = N.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.frei_version() == 20000
    assert lib.frei_last_error() == b""


def test_ctypes_signatures_cover_header():
    from frei_amd import _native as N
    assert set(_declared()) == set(N.SIGNATURES)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from frei_amd import _native as N
    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        N.lib()


def test_argument_errors_without_gpu():
    """Validation happens before any device call, so it is testable on CPU."""
    import ctypes
    from frei_amd import _native as N
    lib = N.lib()
    ctx = ctypes.c_void_p()
    assert lib.frei_ctx_create(ctypes.byref(ctx), 0, 2, 100, 1) != 0
    assert b"n_layers" in lib.frei_last_error()
    assert lib.frei_ctx_create(ctypes.byref(ctx), 0, 30, 1, 1) != 0
    assert lib.frei_sweep(None, 0, 1.0, None, None, None) != 0


def test_kernel_objects_target_gfx950():
    so = os.path.join(ROOT, "frei_amd", "libfrei_hip.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_binning_argument_errors_without_gpu():
    """frei_xsec_create validates the high-resolution axis before touching a device."""
    import ctypes
    import numpy as np
    from frei_amd import _native as N
    lib = N.lib()
    h = ctypes.c_void_p()
    vals = np.zeros((1, 1, 4), dtype=np.float32)
    T, p = np.array([1000.0]), np.array([1.0])
    wl = np.array([1.0, 2.0, 2.0, 3.0])
    assert lib.frei_xsec_create(ctypes.byref(h), 0, N.fptr(vals), 1, 1, 4, N.dptr(T), N.dptr(p),
                                N.dptr(wl)) != 0
    assert b"ascending" in lib.frei_last_error()
    assert lib.frei_xsec_bin(None, 0, None, None, 0, None, 0, None, 0, None) != 0
