"""ctypes binding of the CPU parity oracle (oracle/build/liboracle_fpm.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and only as the checker
(or the timed CPU baseline); the product path (fastest_image_pattern_matching_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from fastest_image_pattern_matching_amd._lib import Params, Result

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "liboracle_fpm.so")
# -ffast-math build of the same source: bench.py's CPU timing variant only, never a parity checker
ORACLE_LIB_FAST = os.path.join(ORACLE_DIR, "build", "liboracle_fpm_fast.so")
_U8P = C.POINTER(C.c_uint8)
_libs = {}
TRACE_DTYPE = np.dtype([("origin", "<i4"), ("layer", "<i4"), ("n3", "<i4"), ("imax", "<i4"),
                        ("angle", "<f8", 3), ("score", "<f8", 3), ("x", "<f8", 3), ("y", "<f8", 3),
                        ("second", "<f8", 3)])


def load(path: str = ORACLE_LIB):
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        subprocess.check_call(["make", "-C", ORACLE_DIR])
    lib = C.CDLL(path)
    lib.orc_create.restype = C.c_void_p
    lib.orc_destroy.argtypes = [C.c_void_p]
    lib.orc_set_params.argtypes = [C.c_void_p, C.POINTER(Params)]
    lib.orc_get_params.argtypes = [C.c_void_p, C.POINTER(Params)]
    lib.orc_learn.argtypes = [C.c_void_p, _U8P, C.c_int, C.c_int, C.c_size_t]
    lib.orc_match.argtypes = [C.c_void_p, _U8P, C.c_int, C.c_int, C.c_size_t, C.POINTER(Result), C.c_int,
                              C.POINTER(C.c_int), C.POINTER(C.c_double)]
    lib.orc_search_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int]
    lib.orc_candidates.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.orc_top_candidates.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int]
    lib.orc_set_trace.argtypes = [C.c_void_p, C.c_int]
    lib.orc_trace.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int]
    lib.orc_template_info.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.orc_template_level.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                       C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                       C.POINTER(C.c_int), _U8P, C.c_size_t]
    lib.orc_pyr_down.argtypes = [_U8P, C.c_int, C.c_int, C.c_size_t, _U8P, C.c_size_t]
    lib.orc_warp_affine.argtypes = [_U8P, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_double), _U8P, C.c_int,
                                    C.c_int, C.c_size_t, C.c_int]
    lib.orc_rotation_matrix.argtypes = [C.c_float, C.c_float, C.c_double, C.POINTER(C.c_double)]
    lib.orc_ncc_map.argtypes = [C.c_void_p, _U8P, C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_int,
                                C.POINTER(C.c_float)]
    lib.orc_rotrect_overlap.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_double),
                                        C.POINTER(C.c_int)]
    lib.orc_set_ccorr_mode.argtypes = [C.c_void_p, C.c_int]
    lib.orc_cross_corr_f32.argtypes = [_U8P, C.c_int, C.c_int, C.c_size_t, _U8P, C.c_int, C.c_int, C.c_size_t,
                                       C.POINTER(C.c_float)]
    lib.orc_filter_rotated_rect.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int, C.c_double,
                                            C.POINTER(C.c_int32)]
    lib.fpm_params_default.argtypes = [C.POINTER(Params)]
    _libs[path] = lib
    return lib


def _u8(a):
    return a.ctypes.data_as(_U8P)


def pyr_down(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
    load().orc_pyr_down(_u8(img), w, h, img.strides[0], _u8(out), out.strides[0])
    return out


def warp_affine(img: np.ndarray, m, dsize, border: int = 0) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    dw, dh = dsize
    out = np.zeros((dh, dw), np.uint8)
    mm = (C.c_double * 6)(*np.asarray(m, np.float64).ravel().tolist())
    load().orc_warp_affine(_u8(img), w, h, img.strides[0], mm, _u8(out), dw, dh, out.strides[0], int(border))
    return out


def rotation_matrix(cx: float, cy: float, angle: float) -> np.ndarray:
    m = (C.c_double * 6)()
    load().orc_rotation_matrix(cx, cy, angle, m)
    return np.array(m[:], np.float64).reshape(2, 3)


def cross_corr_f32(img: np.ndarray, templ: np.ndarray) -> np.ndarray:
    """TM_CCORR map as OpenCV's crossCorr computes it (float32 DFTs, block structure): the oracle's sensitivity
    mode, not the parity contract."""
    img = np.ascontiguousarray(img, np.uint8)
    templ = np.ascontiguousarray(templ, np.uint8)
    (h, w), (th, tw) = img.shape, templ.shape
    out = np.zeros((h - th + 1, w - tw + 1), np.float32)
    rc = load().orc_cross_corr_f32(_u8(img), w, h, img.strides[0], _u8(templ), tw, th, templ.strides[0],
                                   out.ctypes.data_as(C.POINTER(C.c_float)))
    assert rc == 0
    return out


def filter_rotated_rect(corners, scores, max_overlap):
    """filterWithRotatedRect on rectangles given as (ltx, lty, rtx, rty, rbx, rby) rows with scores, in the given order:
    the indices of the survivors in order."""
    c = np.ascontiguousarray(corners, np.float32).reshape(-1, 6)
    sc = np.ascontiguousarray(scores, np.float64).ravel()
    keep = np.zeros(max(len(sc), 1), np.int32)
    n = load().orc_filter_rotated_rect(c.ctypes.data_as(C.POINTER(C.c_float)), sc.ctypes.data_as(C.POINTER(C.c_double)),
                                       len(sc), float(max_overlap), keep.ctypes.data_as(C.POINTER(C.c_int32)))
    return keep[:n].tolist()


def rotrect_overlap(a, b):
    """(type, area, npts) of two rotated rects given as (ptLT, ptRT, ptRB)."""
    fa = (C.c_float * 6)(*[float(v) for v in np.ravel(a)])
    fb = (C.c_float * 6)(*[float(v) for v in np.ravel(b)])
    area, n = C.c_double(), C.c_int()
    t = load().orc_rotrect_overlap(fa, fb, C.byref(area), C.byref(n))
    return t, area.value, n.value


class OracleMatcher:
    """Same surface as fastest_image_pattern_matching_amd.TemplateMatcher (setters, learnPattern, match)."""

    def __init__(self, lib_path: str = ORACLE_LIB):
        self._lib = load(lib_path)
        self._h = C.c_void_p(self._lib.orc_create())
        self._p = Params()
        self._lib.fpm_params_default(C.byref(self._p))
        self.last_time = 0.0

    def __del__(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.orc_destroy(self._h)
            self._h = None

    @property
    def params(self) -> Params:
        return self._p

    def set(self, **kw):
        for k, v in kw.items():
            setattr(self._p, k, v)
        return self

    def learnPattern(self, t: np.ndarray) -> bool:
        t = np.ascontiguousarray(t, np.uint8)
        self._lib.orc_set_params(self._h, C.byref(self._p))
        return self._lib.orc_learn(self._h, _u8(t), t.shape[1], t.shape[0], t.strides[0]) == 0

    def match_raw(self, s: np.ndarray):
        s = np.ascontiguousarray(s, np.uint8)
        self._lib.orc_set_params(self._h, C.byref(self._p))
        cap = 4096
        out = (Result * cap)()
        n = C.c_int()
        sec = C.c_double(self.last_time)
        rc = self._lib.orc_match(self._h, _u8(s), s.shape[1], s.shape[0], s.strides[0], out, cap, C.byref(n),
                                 C.byref(sec))
        self.last_time = sec.value
        return rc, [tuple(getattr(out[i], f) for f, _ in Result._fields_) for i in range(min(n.value, cap))]

    def match(self, s: np.ndarray):
        return self.match_raw(s)[1]

    def stats(self):
        buf = (C.c_int64 * 64)()
        k = self._lib.orc_search_stats(self._h, buf, 64)
        return list(buf[:k])

    def candidates(self) -> np.ndarray:
        """Candidate records of the last match in push order (fpm_candidate / matcher.CANDIDATE_DTYPE)."""
        from fastest_image_pattern_matching_amd.matcher import CANDIDATE_DTYPE

        n = self._lib.orc_candidates(self._h, None, 0)
        out = np.zeros(n, CANDIDATE_DTYPE)
        if n:
            self._lib.orc_candidates(self._h, out.ctypes.data_as(C.c_void_p), n)
        return out

    def set_ccorr_mode(self, mode: int):
        """TM_CCORR arithmetic of the next searches: 0 = exact integer sum rounded once (parity), 1 = OpenCV's
        float32-DFT crossCorr (sensitivity mode for the reference's screenshots)."""
        assert self._lib.orc_set_ccorr_mode(self._h, int(mode)) == 0
        return self

    def set_trace(self, on: bool = True):
        self._lib.orc_set_trace(self._h, 1 if on else 0)
        return self

    def trace(self) -> np.ndarray:
        """Refinement decisions of the last match (after set_trace): one structured row per (candidate, layer)
        with the candidate's push-order index, the layer, the chosen angle slot and the (angle, score, x, y) of
        each of the up to 3 angles (TemplateMatcher.cpp:279-332), plus the runner-up value of each angle's map."""
        n = self._lib.orc_trace(self._h, None, 0)
        buf = np.zeros((max(n, 1), 19), np.float64)
        self._lib.orc_trace(self._h, buf.ctypes.data_as(C.POINTER(C.c_double)), n)
        buf = buf[:n]
        out = np.zeros(n, TRACE_DTYPE)
        out["origin"], out["layer"], out["n3"], out["imax"] = (buf[:, k].astype(np.int32) for k in range(4))
        for f, k in (("angle", 4), ("score", 5), ("x", 6), ("y", 7), ("second", 8)):
            out[f] = buf[:, k:19:5]
        return out

    def top_candidates(self):
        n = self._lib.orc_top_candidates(self._h, None, 0)
        buf = (C.c_double * (4 * max(n, 1)))()
        self._lib.orc_top_candidates(self._h, buf, n)
        return np.array(buf[:4 * n], np.float64).reshape(n, 4)

    def template_levels(self):
        lv, border = C.c_int(), C.c_int()
        self._lib.orc_template_info(self._h, C.byref(lv), C.byref(border))
        out = []
        for i in range(lv.value):
            w, h, eq = C.c_int(), C.c_int(), C.c_int()
            mean, norm, inv = C.c_double(), C.c_double(), C.c_double()
            self._lib.orc_template_level(self._h, i, C.byref(w), C.byref(h), C.byref(mean), C.byref(norm),
                                         C.byref(inv), C.byref(eq), None, 0)
            px = np.zeros((h.value, w.value), np.uint8)
            self._lib.orc_template_level(self._h, i, C.byref(w), C.byref(h), C.byref(mean), C.byref(norm),
                                         C.byref(inv), C.byref(eq), _u8(px), px.strides[0])
            out.append((px, mean.value, norm.value, inv.value, bool(eq.value)))
        return out, border.value

    def ncc_map(self, img: np.ndarray, layer: int, fold: bool) -> np.ndarray:
        img = np.ascontiguousarray(img, np.uint8)
        levels, _ = self.template_levels()
        th, tw = levels[layer][0].shape
        out = np.zeros((img.shape[0] - th + 1, img.shape[1] - tw + 1), np.float32)
        self._lib.orc_ncc_map(self._h, _u8(img), img.shape[1], img.shape[0], img.strides[0], layer,
                              1 if fold else 0, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out
