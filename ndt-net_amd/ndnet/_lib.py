"""Loader of lib/libndnet_amd.so (the HIP path) with its C-ABI signatures.

The library is built in-tree (``make -C ndt-net_amd`` or
``__graft_entry__.build()``).  There is no fallback: when the library is
missing or no GPU is visible the product entry points raise.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to it

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_PATH = os.environ.get("NDNET_AMD_LIB") or os.path.join(ROOT, "lib", "libndnet_amd.so")  # override: A/B builds (tools/)

NDNET_OK = 0
NDNET_ERR_ARG = -20
NDNET_ERR_HIP = -21
NDNET_ERR_SYNC = -22


class NdtStats(ctypes.Structure):
    """ndnet_ndt_stats (include/ndnet_amd.h)."""
    _fields_ = [
        ("rc", ctypes.c_int32),
        ("prune_rc", ctypes.c_int32),
        ("iters", ctypes.c_uint32),
        ("len", ctypes.c_uint32 * 3),
        ("offset", ctypes.c_double * 3),
        ("voxel_size", ctypes.c_double),
        ("num_nds", ctypes.c_uint64),
        ("num_valid", ctypes.c_uint64),
        ("num_kl", ctypes.c_uint64),
        ("num_events", ctypes.c_uint64),
        ("num_out", ctypes.c_uint64),
    ]


STATS_BYTES = ctypes.sizeof(NdtStats)
assert STATS_BYTES == 96

_lib = None

_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_UL = ctypes.c_ulong
_PUL = ctypes.POINTER(ctypes.c_ulong)
_PU = ctypes.POINTER(ctypes.c_uint)
_PD = ctypes.POINTER(ctypes.c_double)
_PUS = ctypes.POINTER(ctypes.c_ushort)

EXPORTS = {
    # reference ABI (core_legacy/include/ndnet_core/ndt.h, kullback_leibler.h)
    "ndt_downsample": (_I, [_PD, ctypes.c_ushort, _UL, _PU, _PU, _PU, _PD, _PD, _PD, _PD, _PUS, ctypes.c_ushort,
                            _UL, _PD, _PUL, _PD, _PUS, ctypes.POINTER(_P), _PUL, ctypes.POINTER(_P), _PUL]),
    "prune_nds": (_I, [_P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, _UL, _PUL, _P, _PUL]),
    "to_point_cloud": (_I, [_P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_double, ctypes.c_double,
                            ctypes.c_double, ctypes.c_double, _PD, _PUL, _PD, _PUS]),
    "free_nds": (None, [_P, _UL]),
    "free_kl_divergences": (None, [_P]),
    "print_matrix": (None, [_P, _I, _I]),  # matrix.h:40 (host only)
    # batched device API
    "ndnet_ndt_plan_create": (_I, [_I, _U64, _U64, _I, _U64, ctypes.POINTER(_P)]),
    "ndnet_ndt_plan_destroy": (None, [_P]),
    "ndnet_ndt_set_path": (_I, [_P, _I]),
    "ndnet_ndt_get_path": (_I, [_P]),
    "ndnet_ndt_get_front_lanes": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "ndnet_ndt_take_sync_failures": (_I, [_P]),
    "ndnet_ndt_set_cu_share": (_I, [_P, _I, _I]),
    "ndnet_ndt_set_exact_counts": (_I, [_P, _I]),
    "ndnet_ndt_set_front_staged": (_I, [_P, _I]),
    "ndnet_ndt_get_front_staged": (_I, [_P]),
    "ndnet_ndt_set_run_part": (_I, [_P, _I]),
    "ndnet_ndt_set_lazy_list": (_I, [_P, _I]),
    "ndnet_ndt_set_heavy_threshold": (_I, [_P, ctypes.c_uint32]),
    "ndnet_ndt_set_welford_form": (_I, [_P, _I]),
    "ndnet_ndt_get_welford_form": (_I, [_P]),
    "ndnet_ndt_debug_set_sync_timeout": (_I, [_P, ctypes.c_uint64]),
    "ndnet_ndt_run": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "ndnet_ndt_run_f64": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ndnet_ndt_prune": (_I, [_P, _P, _U64, _P, _P, _P, _P, _P, _P]),
    "ndnet_ndt_debug_dump": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ndnet_ndt_debug_set_epoch": (_I, [_P, ctypes.c_uint32]),
    "ndnet_ndt_debug_set_kl_fuse": (_I, [_P, _I]),
    "ndnet_ndt_debug_set_list_sort": (_I, [_P, _I]),
    "ndnet_ndt_debug_get_list_sort": (_I, [_P]),
    "ndnet_ndt_debug_kl_marks": (_I, [_P, _P]),
    "ndnet_ndt_debug_front_marks": (_I, [_P, _P]),
    "ndnet_ndt_debug_wq_marks": (_I, [_P, _P, ctypes.POINTER(ctypes.c_uint32)]),
    "ndnet_debug_lu_chain": (_I, [_P, ctypes.c_uint32, _I, _P, _P, _P, _P]),
    "ndnet_ndt_debug_front_wg_marks": (_I, [_P, _P, ctypes.POINTER(_I)]),
    "ndnet_ndt_set_timing": (_I, [_P, _I]),
    "ndnet_ndt_stage_ms": (_I, [_P, _P]),
    "ndnet_amd_version": (ctypes.c_char_p, []),
}


def lib() -> ctypes.CDLL:
    """The loaded library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {ROOT}` "
                               "(there is no CPU fallback)")
        _lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in {**POINTNET_EXPORTS, **TRAIN_EXPORTS}.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


# include/ndnet_pointnet.h
POINTNET_EXPORTS: dict = {
    "ndnet_pn_chain_run": (_I, [_P, _I, _P]),
    "ndnet_pn_chain_run_t32": (_I, [_P, _I, _P]),
    "ndnet_pn_debug_stamps": (_I, [_P, _I]),
    "ndnet_pn_debug_stamps_clear": (_I, []),
    # include/ndnet_ingest.h (host code: the ASCII-PLY reader)
    "ndnet_ply_count": (_I, [ctypes.c_char_p, _I, ctypes.POINTER(_U64)]),
    "ndnet_ply_read": (_I, [ctypes.c_char_p, _I, _I, _P, _P, _U64, ctypes.POINTER(_U64), _I]),
    "ndnet_pn_fc_run": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "ndnet_pn_fc_mfma_run": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "ndnet_pn_head3_run": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ndnet_pn_fold_t2_run": (_I, [_P, _I, _P, _P, _I, _P, _P, _I, _P]),
    "ndnet_pn_fold_prepare": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int64)]),
    "ndnet_pn_fold_run": (_I, [_P, _I, ctypes.c_int64, _P]),
}


_I64 = ctypes.c_int64

# include/ndnet_train.h
TRAIN_EXPORTS: dict = {
    "ndnet_tr_gemm": (_I, [_P, _P, _P, _P, _I64, _I, _I, _I, _I64, _I64, _I64, _I64, _I64, _I64, _I, _I, _I, _I, _I,
                           _I, _P]),
    "ndnet_tr_sum_parts": (_I, [_P, _P, _I64, _I, _P]),
    "ndnet_tr_sum_parts_2d": (_I, [_P, _P, _I64, _I64, _I64, _I, _P]),
    "ndnet_tr_bn_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, ctypes.c_float, ctypes.c_float, _I, _P, _P,
                             _P, _P]),
    "ndnet_tr_bn_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "ndnet_tr_chan_sum": (_I, [_P, _P, _I, _I, _I, _P]),
    "ndnet_tr_row_sum": (_I, [_P, _P, _I64, _I, _P]),
    "ndnet_tr_argmax_match": (_I, [_P, _P, _I64, _I, _P, _P]),
    "ndnet_tr_argmax_match_cm": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "ndnet_row_argmax": (_I, [_P, _I64, _I, _P, _P]),
    "ndnet_tr_fc_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I64, ctypes.c_float,
                             ctypes.c_float, _I, _I, _P, _P]),
    "ndnet_tr_fc_bwd_w": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I64, _I, _P]),
    "ndnet_tr_fc_bwd_x": (_I, [_P, _P, _P, _P, _I, _I, _I, _I64, _I, _P]),
    "ndnet_tr_point_transform": (_I, [_P, _P, _I, _P, _I, _P, _I, _I, _P]),
    "ndnet_tr_point_transform_bwd": (_I, [_P, _P, _I, _P, _I, _P, _I, _I, _P]),
    "ndnet_tr_log_softmax_c": (_I, [_P, _P, _I, _I, _I, _P]),
    "ndnet_tr_log_softmax_c_bwd": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "ndnet_tr_nll_onehot": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "ndnet_tr_nll_onehot_bwd": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "ndnet_tr_adam": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.c_double, ctypes.c_float,
                           ctypes.c_float, _P]),
}


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("ndnet_amd needs a ROCm GPU (gfx950); none is visible and there is no CPU fallback")


def check(rc: int, what: str) -> None:
    if rc != NDNET_OK:
        raise RuntimeError(f"{what} failed with code {rc}")


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
