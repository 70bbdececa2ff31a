"""Helpers for multi-process tests that put several ranks on ONE GPU (test infrastructure).

Ranks sharing a device must not have identical device virtual-address layouts: with two
processes that allocate the same buffer sequence (same virtual addresses) running kernels
concurrently on one MI355X, values read through the per-CU caches were intermittently wrong
(different on every run; 1-process runs are bit-reproducible).  Shifting each rank's
allocations by a dummy allocation of its own size made every such run correct and
bit-reproducible.  One process per GPU — the production layout — never shares
a device, so only these tests need it.
"""
import ctypes
import os
import socket

_KEEP = []


def offset_device_allocations(rank, device=0, step_mib=1536):
    """Allocate (and keep) rank * step_mib MiB on ``device`` before the rank's engine."""
    if rank <= 0 or os.environ.get("FREI_TEST_NO_VA_OFFSET") == "1":
        return
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(device) == 0
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(rank * step_mib << 20)) == 0
    _KEEP.append(p)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
