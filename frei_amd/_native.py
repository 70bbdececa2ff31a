"""ctypes binding of the C ABI in include/frei_hip.h (libfrei_hip.so, built in-tree).

There is no CPU fallback: if the shared library is missing or fails to load, every
compute entry point raises ``RuntimeError`` (build it with ``python -m frei_amd.build``
or ``__graft_entry__.build()``).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FREI_HIP_LIB overrides the library path (A/B builds of the same ABI, tools/ab_sweep.py)
_DEFAULT_LIB = os.path.join(_HERE, "libfrei_hip.so")
LIB_PATH = os.environ.get("FREI_HIP_LIB") or _DEFAULT_LIB

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_fp = ctypes.POINTER(ctypes.c_float)

# int (*)(const double* send, double* recv, int64_t n, void* user)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, _dp, _dp, _i64, _vp)

# name -> (restype, argtypes); mirrors include/frei_hip.h exactly
SIGNATURES = {
    "frei_version": (ctypes.c_int, []),
    "frei_last_error": (ctypes.c_char_p, []),
    "frei_device_count": (ctypes.c_int, [_ip]),
    "frei_ctx_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, _i64,
                                       ctypes.c_int]),
    "frei_ctx_destroy": (ctypes.c_int, [_vp]),
    "frei_ctx_create_batch": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int,
                                             _i64, ctypes.c_int, ctypes.c_int]),
    "frei_set_gravity": (ctypes.c_int, [_vp, _dp]),
    "frei_set_ftoa_batch": (ctypes.c_int, [_vp, _dp]),
    "frei_run_batch": (ctypes.c_int, [_vp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_double, _ip, _dp, _dp]),
    "frei_set_grid": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, ctypes.c_double,
                                     ctypes.c_double]),
    "frei_set_table": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, ctypes.c_int, _dp,
                                      ctypes.c_int]),
    "frei_set_table_separable": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _dp,
                                                ctypes.c_double, ctypes.c_double, _dp,
                                                ctypes.c_int, _dp, ctypes.c_int]),
    "frei_set_mmr": (ctypes.c_int, [_vp, _dp]),
    "frei_set_chemistry": (ctypes.c_int, [_vp, _dp, _dp, ctypes.c_int, _dp, ctypes.c_int]),
    "frei_set_fluxes": (ctypes.c_int, [_vp, _dp, _dp]),
    "frei_get_fluxes": (ctypes.c_int, [_vp, _dp, _dp]),
    "frei_get_spectrum": (ctypes.c_int, [_vp, _dp]),
    "frei_set_temperatures": (ctypes.c_int, [_vp, _dp]),
    "frei_get_temperatures": (ctypes.c_int, [_vp, _dp]),
    "frei_sweep": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, _dp, _dp, _dp]),
    "frei_run": (ctypes.c_int, [_vp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                ctypes.c_double, _ip, _dp, _dp, _dp, _dp]),
    "frei_state_init": (ctypes.c_int, [_vp, _dp]),
    "frei_iterate": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_double]),
    "frei_synchronize": (ctypes.c_int, [_vp]),
    "frei_kappa": (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_double, _dp, _dp]),
    "frei_propagate_fluxes": (ctypes.c_int, [ctypes.c_int, _i64, _dp, _dp, _dp, _dp,
                                             ctypes.c_double, ctypes.c_double, _dp, _dp, _dp,
                                             _dp, _dp]),
    "frei_comm_unique_id": (ctypes.c_int, [_vp]),
    "frei_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp]),
    "frei_comm_p2p_handle": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp]),
    "frei_comm_p2p_open": (ctypes.c_int, [_vp, _vp]),
    "frei_comm_init_host": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                           "ALLGATHER_FN", _vp]),
    "frei_ctx_path": (ctypes.c_int, [_vp, _ip]),
    "frei_milne_pressure": (ctypes.c_int, [_vp, _dp, _dp, _dp]),
    "frei_contribution": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, ctypes.c_double, _dp]),
    "frei_set_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int]),
    "frei_setup_timing": (ctypes.c_int, [_vp, _dp]),
    "frei_contract_timing": (ctypes.c_int, [_vp, _dp, _dp]),
    "frei_graph_info": (ctypes.c_int, [_vp, _ip, _ip]),
    "frei_chain_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "frei_tail_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "frei_comm_shared_device": (ctypes.c_int, [_vp, ctypes.c_int]),
    "frei_device_pci_bus_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "frei_timing_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "frei_timing_read": (ctypes.c_int, [_vp, _dp, _ip]),
    "frei_timing_read_exchange": (ctypes.c_int, [_vp, _dp, _ip]),
    "frei_xsec_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, _fp, ctypes.c_int,
                                        ctypes.c_int, _i64, _dp, _dp, _dp]),
    "frei_xsec_create_synthetic": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int, _i64, _dp, _dp,
                                                  _dp, ctypes.c_uint64]),
    "frei_xsec_destroy": (ctypes.c_int, [_vp]),
    "frei_xsec_bin": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _i64, _dp, ctypes.c_int, _dp,
                                     ctypes.c_int, _dp]),
    "frei_xsec_timing": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _ip]),
    "frei_set_table_binned": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, _dp, _dp,
                                             _i64, _i64, _dp, ctypes.c_int, _dp,
                                             ctypes.c_int]),
}

_lib = None


def lib():
    """Load libfrei_hip.so (raises RuntimeError if it is absent: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"frei_amd: native library {LIB_PATH} is missing; build it with "
                               "`python -m frei_amd.build` (no CPU fallback exists)")
        if LIB_PATH == _DEFAULT_LIB and os.environ.get("FREI_SKIP_STAMP") != "1":
            from .build import read_stamp, sources_present, stamp_matches
            # without the csrc sources (an installed package) the stamp cannot be verified: the
            # library is loaded as it is; with them, a library built from other sources is refused
            if sources_present() and not stamp_matches(LIB_PATH):
                built_by = (read_stamp(LIB_PATH)[1] or "unknown compiler").splitlines()
                raise RuntimeError(f"frei_amd: {LIB_PATH} was not built from the sources in this "
                                   "tree (its .stamp hash differs; it was built by "
                                   f"{built_by[0] if built_by else '?'}); rebuild with "
                                   "`python -m frei_amd.build`")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in SIGNATURES.items():
            if LIB_PATH != _DEFAULT_LIB and not hasattr(L, name):
                continue  # an older A/B build (FREI_HIP_LIB) may predate an entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = [ALLGATHER_FN if a == "ALLGATHER_FN" else a for a in args]
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().frei_last_error().decode(errors="replace")
        raise RuntimeError(f"frei_hip: {msg}")


def dptr(a):
    """Pointer to a C-contiguous float64 array (or NULL for None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], "need C-contiguous float64"
    return a.ctypes.data_as(_dp)


def fptr(a):
    """Pointer to a C-contiguous float32 array."""
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"], "need C-contiguous float32"
    return a.ctypes.data_as(_fp)


def f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def device_count():
    n = ctypes.c_int(0)
    check(lib().frei_device_count(ctypes.byref(n)))
    return n.value
