"""ctypes binding of the C ABI in include/svgdcpp_amd/svgd_capi.h.

The shared library is built in-tree (``make`` at the repo root, or
``__graft_entry__.build()``).  There is no fallback: if the library is
missing or a symbol is absent, importing the device path raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsvgdcpp_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "svgdcpp_amd", "svgd_capi.h")

SVGD_OK = 0
SVGD_ERR_DIM = -1
SVGD_ERR_UNSET = -2
SVGD_ERR_ARG = -3
SVGD_ERR_HIP = -4
SVGD_ERR_RCCL = -5
SVGD_ERR_RUNTIME = -6

SVGD_F64 = 0
SVGD_F32 = 1
SVGD_OPT_ADAM = 0
SVGD_OPT_ADAGRAD = 1
SVGD_OPT_RMSPROP = 2
SVGD_SCALE_MEDIAN = 0
SVGD_SCALE_FIXED = 2
SVGD_SCALE_MATRIX = 3
SVGD_SCALE_HESSIAN = 1
SVGD_MEDIAN_DIRECT = 0
SVGD_MEDIAN_BRACKET = 1
SVGD_MEDIAN_FALLBACK = 2
SVGD_MEDIAN_REBRACKET = 3
# svgd_get_diagnostics slots (svgd_capi.h SVGD_DIAG_*)
DIAG_NAMES = ("steps", "phi_kernel_ms", "phi_kernel_n", "phi_wait_ms", "phi_wait_n", "coll_ms",
              "coll_n", "gather_g_ms", "gather_g_n", "host_grad_ms", "host_xwait_ms",
              "host_job_ms", "host_wait_ms", "ranks", "host_threads", "trk_steps", "trk_miss",
              "sim_world", "cpu_quota", "split_steps", "mirror_steps", "spec_steps", "g_comm", "trk_band")
SVGD_DIAG_LEN = len(DIAG_NAMES)

_D = ctypes.POINTER(ctypes.c_double)
_I64 = ctypes.c_int64
_P = ctypes.c_void_p

# name -> (restype, argtypes); every function declared in svgd_capi.h
SIGNATURES = {
    "svgd_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int]),
    "svgd_create_dist": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _I64, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    "svgd_create_sim": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int]),
    "svgd_get_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "svgd_destroy": (ctypes.c_int, [_P]),
    "svgd_last_error": (ctypes.c_char_p, [_P]),
    "svgd_shard": (ctypes.c_int, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_set_optimizer": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double]),
    "svgd_reset_optimizer": (ctypes.c_int, [_P]),
    "svgd_set_bounds": (ctypes.c_int, [_P, _D, _D]),
    "svgd_set_scale": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_double]),
    "svgd_set_particles": (ctypes.c_int, [_P, _D]),
    "svgd_get_particles": (ctypes.c_int, [_P, _D]),
    "svgd_get_shard": (ctypes.c_int, [_P, _D]),
    "svgd_median_scale": (ctypes.c_int, [_P, _D, _D]),
    "svgd_phi": (ctypes.c_int, [_P, _D, ctypes.c_double, _D]),
    "svgd_step": (ctypes.c_int, [_P, _D]),
    "svgd_begin_step": (ctypes.c_int, [_P, _D]),
    "svgd_finish_step": (ctypes.c_int, [_P, _D]),
    "svgd_step_host_model": (ctypes.c_int, [_P, ctypes.c_void_p]),
    "svgd_host_buffers": (ctypes.c_int, [_P, ctypes.POINTER(_D), ctypes.POINTER(_D)]),
    "svgd_sync": (ctypes.c_int, [_P]),
    "svgd_last_scale": (ctypes.c_int, [_P, _D, _D, ctypes.POINTER(ctypes.c_int)]),
    "svgd_last_median_keys": (ctypes.c_int, [_P, _D, _D, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "svgd_set_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "svgd_get_timing": (ctypes.c_int, [_P, _D, _D, ctypes.POINTER(_I64)]),
    "svgd_get_diagnostics": (ctypes.c_int, [_P, _D, ctypes.c_int]),
    "svgd_set_median_tuning": (ctypes.c_int, [_P, _I64, _I64, _I64]),
    "svgd_phi_kernel_name": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int]),
    "svgd_debug_pair_keys": (ctypes.c_int, [_P, _D, _I64]),
    "svgd_set_scale_matrix": (ctypes.c_int, [_P, _D]),
    "svgd_set_step_hessian_sum": (ctypes.c_int, [_P, _D]),
    "svgd_get_scale_matrix": (ctypes.c_int, [_P, _D]),
    "svgd_set_device_model": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "svgd_device_logp_grad": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "svgd_plan_rows": (None, [_I64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_plan_median_ranks": (ctypes.c_int, [_I64, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_plan_pair_tiles": (_I64, [_I64, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "svgd_plan_pair_tile": (None, [_I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64, ctypes.POINTER(_I64),
                                   ctypes.POINTER(_I64)]),
    "svgd_plan_sym_units": (_I64, [_I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int),
                                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_plan_sym_total": (_I64, [_I64, ctypes.c_int, ctypes.c_int]),
    "svgd_plan_sym_unit": (ctypes.c_int, [_I64, ctypes.c_int, ctypes.c_int, _I64, ctypes.POINTER(_I64),
                                          ctypes.POINTER(_I64)]),
    "svgd_plan_sym_exchange": (None, [_I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_plan_bucket_select": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "svgd_model_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.c_int, _D, _D]),
    "svgd_model_destroy": (ctypes.c_int, [_P]),
    "svgd_model_logp_grad": (ctypes.c_int, [_P, _D, _I64, _D]),
    "svgd_model_neg_hess_sum": (ctypes.c_int, [_P, _D, _I64, _D]),
}

_lib = None


def lib():
    """Load libsvgdcpp_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"svgdcpp_amd: {LIB_PATH} is missing -- run `make` (or "
                              "__graft_entry__.build()); there is no CPU fallback")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name)  # AttributeError if the symbol is missing
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def dptr(a):
    """double* of a C-contiguous float64 numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(_D)
