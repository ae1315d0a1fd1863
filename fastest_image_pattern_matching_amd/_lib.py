"""ctypes binding of libfpm_hip.so (include/fpm.h).

The shared library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()`` or ``make -C
fastest_image_pattern_matching_amd/csrc``).  There is no CPU fallback: if the library is missing or no gfx950
device is present, loading / context creation raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libfpm_hip.so")
CSRC = os.path.join(_HERE, "csrc")

FPM_OK = 0
FPM_E_INVALID_ARG = -1
FPM_E_NOT_LEARNED = -2
FPM_E_SIZE = -3
FPM_E_DEVICE = -4
FPM_E_CAPACITY = -5
FPM_E_INTERNAL = -6

(K_PYR, K_TOP_WARP, K_TOP_NCC, K_TOP_NMS, K_CAND_INIT, K_ROI_TABLES, K_ROI_WARP, K_ROI_CORR, K_ROI_EVAL, K_ROI_SMALL,
 K_CAND_STEP, K_TOP_MAP) = range(12)
# profiling index -> kernel (include/fpm.h FPM_K_*); top_ncc is k_top_mma (matrix-core top layer) where it applies, else
# k_ncc_tile for templates up to 128 x 64; top_map = k_top_map, the matrix-core form's fallback (full maps for the jobs
# its lists left)
KERNEL_NAMES = ["pyr_down", "top_warp", "top_ncc", "top_nms", "cand_init", "roi_tables", "roi_warp", "roi_corr",
                "roi_eval", "roi_small", "cand_step", "top_map"]
KERNEL_SYMBOLS = {"pyr_down": ["k_pyr_down_s", "k_pyr_down"], "top_warp": ["k_warp"],
                  "top_ncc": ["k_top_mma", "k_ncc_tile", "k_ncc_map"],
                  "top_nms": ["k_nms_greedy", "k_nms"], "cand_init": ["k_cand_init"], "roi_tables": ["k_roi_tables"],
                  "roi_warp": ["k_roi_warp3", "k_roi_warp"], "roi_corr": ["k_roi_corr"], "roi_eval": ["k_roi_eval"],
                  "roi_small": ["k_roi_small"], "cand_step": ["k_cand_step"], "top_map": ["k_top_map"]}


class Params(C.Structure):
    """fpm_params — the 7 TemplateMatcher setters + hidden range members (TemplateMatcher.h:22-28, 88-89)."""

    _fields_ = [
        ("max_pos", C.c_int32),
        ("min_reduce_area", C.c_int32),
        ("max_overlap", C.c_double),
        ("score", C.c_double),
        ("tolerance_angle", C.c_double),
        ("use_simd", C.c_int32),
        ("subpixel", C.c_int32),
        ("tolerance_range", C.c_int32),
        ("semantics", C.c_int32),
        ("tolerance", C.c_double * 4),
        ("top_angle_step", C.c_double),
    ]


class Result(C.Structure):
    """fpm_result — POD-identical to s_SingleTargetMatch (DataStructures.h:97-115)."""

    _fields_ = [(n, C.c_double) for n in (
        "lt_x", "lt_y", "rt_x", "rt_y", "rb_x", "rb_y", "lb_x", "lb_y", "cx", "cy", "angle", "score")]


class Candidate(C.Structure):
    """fpm_candidate — one top-layer candidate (s_MatchParameter, DataStructures.h:58-94) and its refinement."""

    _fields_ = [("top_score", C.c_double), ("x", C.c_double), ("y", C.c_double), ("score", C.c_double),
                ("angle", C.c_double), ("angle_index", C.c_int32), ("peak_rank", C.c_int32), ("source", C.c_int32),
                ("kept", C.c_int32)]


# every symbol include/fpm.h declares, with (restype, argtypes)
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
SIGNATURES = {
    "fpm_params_default": (None, [C.POINTER(Params)]),
    "fpm_abi_version": (C.c_int, []),
    "fpm_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "fpm_destroy": (C.c_int, [_P]),
    "fpm_last_error": (C.c_char_p, [_P]),
    "fpm_set_params": (C.c_int, [_P, C.POINTER(Params)]),
    "fpm_get_params": (C.c_int, [_P, C.POINTER(Params)]),
    "fpm_learn": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t]),
    "fpm_clear_pattern": (C.c_int, [_P]),
    "fpm_is_learned": (C.c_int, [_P]),
    "fpm_match": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t, C.POINTER(Result), C.c_int32,
                            C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
    "fpm_stage_sources": (C.c_int, [_P, C.POINTER(_U8P), C.c_int32, C.c_int32, C.c_int32, C.c_size_t]),
    "fpm_match_staged": (C.c_int, [_P, C.POINTER(Result), C.c_int32, C.POINTER(C.c_int32)]),
    "fpm_match_staged_launch": (C.c_int, [_P]),
    "fpm_match_staged_finish": (C.c_int, [_P, C.POINTER(Result), C.c_int32, C.POINTER(C.c_int32)]),
    "fpm_op_pyr_down": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t, _U8P, C.c_size_t]),
    "fpm_op_pyr_down2": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t, _U8P, C.c_size_t, _U8P, C.c_size_t,
                                   C.c_int32, C.c_int32]),
    "fpm_op_warp_affine": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t, C.POINTER(C.c_double), _U8P,
                                     C.c_int32, C.c_int32, C.c_size_t, C.c_int32]),
    "fpm_op_ncc_map": (C.c_int, [_P, _U8P, C.c_int32, C.c_int32, C.c_size_t, C.c_int32, C.c_int32,
                                 C.POINTER(C.c_float)]),
    "fpm_op_overlap_filter": (C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int32, C.c_double,
                                        C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "fpm_template_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "fpm_template_level": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                     C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_int32), _U8P, C.c_size_t]),
    "fpm_set_angle_shard": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "fpm_get_angle_shard": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "fpm_last_candidates": (C.c_int, [_P, C.c_int32, C.POINTER(Candidate), C.c_int32, C.POINTER(C.c_int32)]),
    "fpm_last_results": (C.c_int, [_P, C.POINTER(Result), C.c_int32, C.POINTER(C.c_int32)]),
    "fpm_merge_candidates": (C.c_int, [C.POINTER(Params), C.c_int32, C.c_int32, C.POINTER(Candidate), C.c_int32,
                                       C.POINTER(Result), C.c_int32, C.POINTER(C.c_int32)]),
    "fpm_search_stats": (C.c_int, [_P, C.POINTER(C.c_int64), C.c_int32]),
    "fpm_search_bytes": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "fpm_profile_enable": (C.c_int, [_P, C.c_int32]),
    "fpm_profile_reset": (C.c_int, [_P]),
    "fpm_profile_get": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                  C.POINTER(C.c_int64)]),
    "fpm_profile_last": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
}

_lib = None


def build_library(force: bool = False) -> str:
    """Compile libfpm_hip.so in-tree with hipcc for gfx950 (no-op when up to date)."""
    cmd = ["make", "-C", CSRC, "-j8"]
    if force:
        subprocess.check_call(["make", "-C", CSRC, "clean"])
    subprocess.check_call(cmd)
    return LIB_PATH


def load(build_if_missing: bool = True) -> C.CDLL:
    """Load libfpm_hip.so; raises if it cannot be built or loaded (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing:
            raise RuntimeError(f"{LIB_PATH} not built; run make -C {CSRC}")
        build_library()
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def u8ptr(a):
    return a.ctypes.data_as(_U8P)
