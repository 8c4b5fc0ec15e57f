"""Loader and ctypes bindings for libsts_hip.so (the C ABI in include/sts.h).

This is the Python analogue of the JNI shim: plain pointers and
sizes cross the boundary, no torch types.  There is deliberately NO fallback:
if the HIP library is missing or no gfx950 device is visible, every operator
raises -- the product path never computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
# The product library is the in-tree build; the package reads no environment variable (an
# executor's environment must not be able to swap the library).  Measurement tools select
# another build explicitly with use_library() before the first call.
LIB_PATH = os.path.join(PKG_ROOT, "build", "libsts_hip.so")

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_vp = ctypes.c_void_p
_c_dbl = ctypes.c_double

# name -> (restype, argtypes); mirrors include/sts.h exactly (tests/test_abi.py checks
# that every symbol declared there is exported and bound here).
SIGNATURES = {
    "sts_abi_version": (_c_int, []),
    "sts_init": (_c_int, [_c_int]),
    "sts_last_error": (ctypes.c_char_p, []),
    "sts_fill_method_from_name": (_c_int, [ctypes.c_char_p]),
    "sts_stream_synchronize": (_c_int, [_c_vp]),
    "sts_profile_begin": (_c_int, []),
    "sts_profile_end": (_c_int, [_c_vp, _c_vp]),
    "sts_fill": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_vp, _c_vp]),
    "sts_diff_at_lag": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp]),
    "sts_lag_matrix": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp]),
    "sts_autocorr": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_vp, _c_vp]),
    "sts_ewma_add": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_ewma_remove": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_ar_fit": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_ar_rule_count": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp]),
    "sts_ar_remove": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp]),
    "sts_ar_add": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp]),
    "sts_fill_autocorr": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    "sts_fill_diff_ewma": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    "sts_fill_lag_matrix": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_int,
                                     _c_vp, _c_vp]),
    "sts_ar_fit_remove": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp,
                                   _c_vp, _c_vp]),
    "sts_ewma_fit": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp]),
    "sts_ewma_sse_gradient": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_garch_fit": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp]),
    "sts_garch_loglik_gradient": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_garch_remove": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_garch_add": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_argarch_remove": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64] + [_c_vp] * 6),
    "sts_argarch_add": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64] + [_c_vp] * 6),
    "sts_argarch_fit": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_series_stats": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_nan_instants": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_active_instants": (_c_int, [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp]),
    "sts_gather_instants": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp]),
    "sts_to_instants": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp]),
    "sts_wire_scan": (_c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_wire_decode": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp]),
    "sts_wire_encode": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp]),
    "sts_observations_to_panel": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp]),
    "sts_csv_parse": (_c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64]),
    "sts_arima_fit_ar": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_gen_panel": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_uint64, _c_dbl, _c_vp]),
    "sts_gen_ar_panel": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_uint64, _c_int, _c_vp]),
    "sts_fill_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_vp]),
    "sts_autocorr_host": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_vp]),
    "sts_diff_at_lag_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int]),
    "sts_lag_matrix_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int]),
    "sts_ewma_add_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp]),
    "sts_ewma_remove_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp]),
    "sts_ewma_fit_host": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_garch_fit_host": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp]),
    "sts_argarch_fit_host": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
    "sts_ar_fit_host": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    "sts_ar_remove_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_int]),
    "sts_ar_add_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_int]),
    "sts_host_alloc": (_c_int, [ctypes.c_size_t, _c_vp]),
    "sts_host_free": (_c_int, [_c_vp]),
    "sts_staging_release": (_c_int, []),
    "sts_staging_stats": (_c_int, [_c_vp]),
    "sts_staging_set_limit": (_c_int, [_c_int]),
    "sts_staging_pool_info": (_c_int, [_c_vp]),
    "sts_fill_autocorr_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp]),
    "sts_fill_diff_ewma_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp]),
    "sts_ar_fit_remove_host": (_c_int, [_c_vp, _c_vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp]),
}

_lib = None
_lock = threading.Lock()
_inited = set()


class NativeLibraryError(RuntimeError):
    """libsts_hip.so is missing or unusable: there is no CPU fallback."""


def load_library(path: str = LIB_PATH):
    """Load and bind libsts_hip.so (no device needed, used by the CPU ABI tests)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise NativeLibraryError(
                    "libsts_hip.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (there is no CPU fallback)" % path)
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def lib():
    return load_library()


def use_library(path: str) -> None:
    """Bind the process to ANOTHER build of the library (same C ABI) before its first use:
    bench.py / tools/ pass their STS_HIP_LIB here for same-box A/B runs of tools/variant.sh
    builds.  Not called by the product path."""
    global _lib
    with _lock:
        if _lib is not None:
            raise NativeLibraryError("use_library(%s): a library is already loaded" % path)
    v = load_variant(path)
    with _lock:
        _lib = v


_variants = {}


def load_variant(path: str):
    """Bind ANOTHER build of the library (same C ABI) without touching the product handle:
    build/libsts_hip_ab.so (A/B experiment knobs, -DSTS_AB) for the knob parity tests and
    tools/.  The product library never reads its environment."""
    with _lock:
        if path not in _variants:
            if not os.path.exists(path):
                raise NativeLibraryError("library variant not found at %s" % path)
            v = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(v, name)
                fn.restype = res
                fn.argtypes = args
            _variants[path] = v
    return _variants[path]


AB_LIB_PATH = os.path.join(PKG_ROOT, "build", "libsts_hip_ab.so")


def ensure_device(device: int) -> None:
    """sts_init(device) once per (thread, device): selects the HIP device and checks gfx950."""
    key = (threading.get_ident(), device)
    if key in _inited:
        return
    from .errors import raise_for_status
    raise_for_status(lib().sts_init(device), "sts_init")
    _inited.add(key)
