"""ctypes binding of libdwhmc.so (include/dwhmc.h).

This is the Python analogue of the Julia `ccall` layer in INTEGRATION.md: plain
pointers and sizes, no torch types.  Error codes become exceptions the way
the reference's Julia code raises (ArgumentError -> ValueError, LAPACK/device
failures -> RuntimeError).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import build as _build

DWH_OK = 0
DWH_ERR_ARG = -1
DWH_ERR_HIP = -2
DWH_ERR_STATE = -3
DWH_ERR_SPECTRUM = -4
DWH_ERR_TABLE = -5


class DwhError(RuntimeError):
    """Device-side failure (no GPU, HIP error, guard trip)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[dwhmc {code}] {msg}")
        self.code = code


class SpectrumGuardError(DwhError):
    """|Δ_ij| left the range the pole set was built for (DWH_ERR_SPECTRUM)."""


class c128(C.Structure):
    _fields_ = [("re", C.c_double), ("im", C.c_double)]


class dwh_info_t(C.Structure):
    _fields_ = [("N", C.c_int64), ("Np", C.c_int64), ("nchains", C.c_int64), ("npoles", C.c_int64),
                ("kappa", C.c_double), ("e_bound", C.c_double), ("err_tanh", C.c_double),
                ("delta_cap", C.c_double), ("device_bytes", C.c_int64), ("algo", C.c_int64),
                ("block", C.c_int64), ("eig_half", C.c_int64),
                ("eig_long_clusters", C.c_int64), ("eig_quat", C.c_int64)]


_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32
_D = C.c_double
_DP = C.POINTER(C.c_double)

# name -> (restype, argtypes); the exact list include/dwhmc.h declares
SIGNATURES = {
    "dwh_create": (C.c_int, [C.POINTER(_P), _I64, _I64, _D, _D, _D, _D, _D, _P, _P, _P, _I32]),
    "dwh_create_batched": (C.c_int, [C.POINTER(_P), _I64, _I64, _D, _D, _D, _D, _D, _P, _P, _I64, _P,
                                     _D, _I32]),
    "dwh_create_ex": (C.c_int, [C.POINTER(_P), _I64, _I64, _D, _D, _D, _D, _D, _P, _P, _I64, _P,
                                _D, _I32, _I32]),
    "dwh_destroy": (None, [_P]),
    "dwh_last_error": (C.c_char_p, [_P]),
    "dwh_info": (C.c_int, [_P, C.POINTER(dwh_info_t)]),
    "dwh_update_pairing": (C.c_int, [_P, _P]),
    "dwh_factorize": (C.c_int, [_P]),
    "dwh_forces": (C.c_int, [_P, _P, _P]),
    "dwh_pairing": (C.c_int, [_P, _P]),
    "dwh_fermion_energy": (C.c_int, [_P, _P]),
    "dwh_hole_trace": (C.c_int, [_P, _P]),
    "dwh_total_energy": (C.c_int, [_P, _D, _P]),
    "dwh_set_state": (C.c_int, [_P, _P, _P]),
    "dwh_get_state": (C.c_int, [_P, _P, _P]),
    "dwh_hmc_sweep": (C.c_int, [_P, _P, _P, _I64, _D, _D, _P, _P]),
    "dwh_hmc_trajectory": (C.c_int, [_P, _P, _I64, _D, _D, _P]),
    "dwh_hmc_finish": (C.c_int, [_P, _P]),
    "dwh_load_draws": (C.c_int, [_P, _I64, _P, _P]),
    "dwh_run_sweeps": (C.c_int, [_P, _I64, _I64, _I64, _D, _D]),
    "dwh_sweep_results": (C.c_int, [_P, _I64, _I64, _P, _P]),
    "dwh_synchronize": (C.c_int, [_P]),
    "dwh_stream": (C.c_int, [_P, C.POINTER(_P)]),
    "dwh_timing_enable": (C.c_int, [_P, _I32]),
    "dwh_timing_read": (C.c_int, [_P, C.c_char_p, _DP, C.POINTER(_I64), _DP]),
    "dwh_timing_reset": (C.c_int, [_P]),
    "dwh_bench_assembly": (C.c_int, [_P, _I64]),
    "dwh_debug_cr_stamps": (C.c_int, [_P, _I32, _P, _I64]),
    "dwh_eigensystem": (C.c_int, [_P, _I64, _P, _P]),
    "dwh_transport_grid": (C.c_int, [_D, _D, _D, C.POINTER(_I64), C.POINTER(_I64)]),
    "dwh_measure_transport": (C.c_int, [_P, _I64, _D, _D, _D, _DP, _DP, _P, _I64, _P, _P, _I64, _P]),
    "dwh_measure_transport_batched": (C.c_int, [_P, _D, _D, _D, _P, _P, _P, _I64, _P, _P, _I64, _P]),
    "dwh_measure_transport_deltas": (C.c_int, [_P, _I64, _I64, _P, _D, _D, _D, _P, _P, _P, _I64, _P, _P, _I64,
                                               _P]),
    "dwh_debug_dense_H": (C.c_int, [_P, _I64, _P]),
    "dwh_debug_qeig": (C.c_int, [_P, _I64, _P, _P]),
    "dwh_debug_level0": (C.c_int, [_P, _I64, _I64, _I32, _P, _P]),
    "dwh_debug_cr_plan_check": (C.c_int, [_I64, _I64, _I64, _I32, _I32, _P]),
    "dwh_debug_cr_plan_flops": (C.c_int, [_I64, _I64, _I64, _I32, _I32, _P]),
    "dwh_debug_h_bound": (C.c_int, [_I64, _I64, _D, _D, _D, _P, _P, _I64, _P, _P]),
    "dwh_selftest_mfma": (C.c_int, [_I32]),
    "dwh_debug_gemm": (C.c_int, [_I32, _I32, C.c_char, C.c_char, _I64, _I64, _I64, _P, _P, _I64, _P, _I64, _P,
                                 _P, _I64, _I64]),
}

_lib = None


def load(build_if_missing: bool = True) -> C.CDLL:
    """Load (building first if needed) the in-tree libdwhmc.so."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("DWHMC_LIB")   # A/B builds of kernel variants (tools/)
    if path is None:
        if build_if_missing and _build.needs_build():
            _build.build()
        path = _build.LIB
    if not os.path.exists(path):
        raise DwhError(DWH_ERR_HIP, f"{path} missing: run __graft_entry__.build()")
    _lib = load_path(path)
    return _lib


_variants: dict = {}


def load_path(path: str) -> C.CDLL:
    """Load a specific build of the library (A/B variants in tools/)."""
    path = os.path.abspath(path)
    if path not in _variants:
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                # an older build (A/B against an earlier round's library):
                # the entry is missing there, and calling it says so
                if path == os.path.abspath(_build.LIB):
                    raise
                continue
            fn.restype = res
            fn.argtypes = args
        _variants[path] = lib
    return _variants[path]


def lib_path() -> str:
    return _build.LIB


def check(code: int, ctx=None) -> None:
    if code == DWH_OK:
        return
    msg = load().dwh_last_error(ctx).decode(errors="replace")
    if code == DWH_ERR_ARG:
        raise ValueError(msg)
    if code == DWH_ERR_SPECTRUM:
        raise SpectrumGuardError(code, msg)
    raise DwhError(code, msg)


def ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays crossing the C ABI must be contiguous"
    return a.ctypes.data_as(C.c_void_p)
