"""Python mirror of the reference's ``TemplateMatcher`` (include/TemplateMatcher.h:9-90) over the C ABI.

Same method names, argument meaning and error behaviour as the C++ class: ``learnPattern`` returns False on an
empty image (TemplateMatcher.cpp:47-49); ``match`` returns an empty list on an empty source, an unlearned
template or a size mismatch (:99-114); ``getLastExecutionTime`` keeps its previous value when a search finds
nothing (:398-404).  All pixel work runs in libfpm_hip.so on a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib as L


@dataclass
class SingleTargetMatch:
    """s_SingleTargetMatch (DataStructures.h:97-115)."""

    ptLT: Tuple[float, float]
    ptRT: Tuple[float, float]
    ptRB: Tuple[float, float]
    ptLB: Tuple[float, float]
    ptCenter: Tuple[float, float]
    dMatchedAngle: float
    dMatchScore: float

    @staticmethod
    def from_c(r: "L.Result") -> "SingleTargetMatch":
        return SingleTargetMatch((r.lt_x, r.lt_y), (r.rt_x, r.rt_y), (r.rb_x, r.rb_y), (r.lb_x, r.lb_y),
                                 (r.cx, r.cy), r.angle, r.score)

    @staticmethod
    def from_row(r) -> "SingleTargetMatch":
        v = [float(x) for x in r]
        return SingleTargetMatch((v[0], v[1]), (v[2], v[3]), (v[4], v[5]), (v[6], v[7]), (v[8], v[9]), v[10], v[11])

    def getCenterQPoint(self):
        return self.ptCenter

    def getBoundingRect(self):
        xs = [self.ptLT[0], self.ptRT[0], self.ptRB[0], self.ptLB[0]]
        ys = [self.ptLT[1], self.ptRT[1], self.ptRB[1], self.ptLB[1]]
        return (min(xs), min(ys), max(xs) - min(xs), max(ys) - min(ys))

    def as_tuple(self):
        return (*self.ptLT, *self.ptRT, *self.ptRB, *self.ptLB, *self.ptCenter, self.dMatchedAngle,
                self.dMatchScore)


# fpm_candidate as a numpy record (include/fpm.h), 56 bytes
CANDIDATE_DTYPE = np.dtype([("top_score", "<f8"), ("x", "<f8"), ("y", "<f8"), ("score", "<f8"), ("angle", "<f8"),
                            ("angle_index", "<i4"), ("peak_rank", "<i4"), ("source", "<i4"), ("kept", "<i4")])
assert CANDIDATE_DTYPE.itemsize == C.sizeof(L.Candidate)


def merge_candidates(params: "L.Params", tmpl_w: int, tmpl_h: int, cands: np.ndarray) -> List[SingleTargetMatch]:
    """fpm_merge_candidates: the coupled tail of TemplateMatcher::match (TemplateMatcher.cpp:214, 262-432) over one
    source's candidate records in push order (all shards concatenated in shard order).  Host only (no device)."""
    lib = L.load()
    c = np.ascontiguousarray(cands, CANDIDATE_DTYPE)
    cap = max(16, len(c))
    out = (L.Result * cap)()
    n = C.c_int32()
    rc = lib.fpm_merge_candidates(C.byref(params), int(tmpl_w), int(tmpl_h),
                                  c.ctypes.data_as(C.POINTER(L.Candidate)), len(c), out, cap, C.byref(n))
    if rc != L.FPM_OK:
        raise ValueError(f"fpm_merge_candidates failed with {rc} (records not in push order?)")
    return [SingleTargetMatch.from_c(out[i]) for i in range(n.value)]


def _gray(img) -> np.ndarray:
    a = np.asarray(img)
    if a.ndim != 2 or a.dtype != np.uint8:
        raise TypeError("expected a 2-D uint8 (CV_8UC1) image")
    return np.ascontiguousarray(a)


class TemplateMatcher:
    """Drop-in for the reference TemplateMatcher, one context (one HIP stream) per instance."""

    def __init__(self, device: int = 0):
        self._lib = L.load()
        self._ctx = C.c_void_p()
        rc = self._lib.fpm_create(device, C.byref(self._ctx))
        if rc != L.FPM_OK:
            raise RuntimeError(f"fpm_create(device={device}) failed with {rc}: no gfx950 device / HIP runtime")
        self._params = L.Params()
        self._lib.fpm_params_default(C.byref(self._params))
        self._last_time = 0.0
        self._user_rect = None
        self._cap = 64                 # results per source; grown on FPM_E_CAPACITY
        self._staged = 0               # sources of the last stage() (0 after a plain match())
        self._bufs = None              # reusable ctypes result buffers for match_staged

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            self._lib.fpm_destroy(ctx)
            self._ctx = None

    # -- error plumbing ---------------------------------------------------------------------------------
    def last_error(self) -> str:
        s = self._lib.fpm_last_error(self._ctx)
        return s.decode() if s else ""

    def _check(self, rc: int, what: str):
        if rc == L.FPM_E_DEVICE or rc == L.FPM_E_INTERNAL:
            raise RuntimeError(f"{what}: device error {rc}: {self.last_error()}")
        return rc

    def _push(self):
        self._lib.fpm_set_params(self._ctx, C.byref(self._params))

    # -- template -----------------------------------------------------------------------------------------
    def learnPattern(self, templateImage) -> bool:
        a = np.asarray(templateImage)
        if a.size == 0:
            return False
        g = _gray(a)
        self._push()
        rc = self._check(self._lib.fpm_learn(self._ctx, L.u8ptr(g), g.shape[1], g.shape[0], g.strides[0]),
                         "learnPattern")
        return rc == L.FPM_OK

    def isPatternLearned(self) -> bool:
        return bool(self._lib.fpm_is_learned(self._ctx))

    def clearPattern(self):
        self._lib.fpm_clear_pattern(self._ctx)

    # -- search ---------------------------------------------------------------------------------------------
    def match(self, sourceImage) -> List[SingleTargetMatch]:
        a = np.asarray(sourceImage)
        self._staged = 0   # fpm_match replaces a staged batch (fpm_match_staged_launch then fails loudly)
        if a.size == 0 or not self.isPatternLearned():
            # an argument-less fpm_match fails its checks and drops the previous search's candidate records
            self._lib.fpm_match(self._ctx, None, 0, 0, 0, None, 0, C.byref(C.c_int32()), None)
            return []
        g = _gray(a)
        self._push()
        out = (L.Result * self._cap)()
        n = C.c_int32()
        sec = C.c_double(self._last_time)
        rc = self._check(self._lib.fpm_match(self._ctx, L.u8ptr(g), g.shape[1], g.shape[0], g.strides[0], out,
                                             self._cap, C.byref(n), C.byref(sec)), "match")
        if rc == L.FPM_E_CAPACITY:   # fetch the results already computed into a larger buffer (no second search)
            self._cap = max(self._cap * 2, n.value)
            out = (L.Result * self._cap)()
            rc = self._check(self._lib.fpm_last_results(self._ctx, out, self._cap, C.byref(n)), "last_results")
        if rc != L.FPM_OK:
            return []
        self._last_time = sec.value
        return [SingleTargetMatch.from_c(out[i]) for i in range(n.value)]

    def match_batch(self, sources: Sequence[np.ndarray]) -> List[List[SingleTargetMatch]]:
        """Extension: all sources (same size) searched in one device pass (fpm_stage_sources + fpm_match_staged)."""
        self.stage(sources)
        return self.match_staged()

    def stage(self, sources: Sequence[np.ndarray]):
        gs = [_gray(s) for s in sources]
        h, w = gs[0].shape
        if any(g.shape != (h, w) for g in gs):
            raise ValueError("all staged sources must have the same size")
        self._push()
        ptrs = (L._U8P * len(gs))(*[L.u8ptr(g) for g in gs])
        rc = self._check(self._lib.fpm_stage_sources(self._ctx, ptrs, len(gs), w, h, gs[0].strides[0]), "stage")
        if rc != L.FPM_OK:
            raise ValueError(f"fpm_stage_sources failed with {rc}: {self.last_error()}")
        self._staged = len(gs)

    def match_staged(self) -> List[List[SingleTargetMatch]]:
        counts, res = self.match_staged_array()
        return [[SingleTargetMatch.from_row(res[s, i]) for i in range(counts[s])] for s in range(len(counts))]

    def _views(self, n_src):
        if self._bufs is None or self._bufs[0] != (n_src, self._cap):
            out = (L.Result * (self._cap * n_src))()
            n = (C.c_int32 * n_src)()
            views = (np.frombuffer(n, dtype=np.int32), np.frombuffer(out, dtype=np.float64).reshape(n_src, self._cap, 12))
            self._bufs = ((n_src, self._cap), out, n, views)
        return self._bufs

    def match_staged_array(self):
        """Like match_staged, returning (counts[int32, n_src], results[f64, n_src, cap, 12]) views of reused buffers
        (fields in s_SingleTargetMatch order) instead of Python objects; valid until the next call."""
        self.match_staged_launch()
        return self.match_staged_finish_array()

    def match_staged_launch(self):
        """Enqueue the device pass over the staged sources and return (fpm_match_staged_launch)."""
        self._push()
        rc = self._check(self._lib.fpm_match_staged_launch(self._ctx), "match_staged_launch")
        if rc != L.FPM_OK:
            raise RuntimeError(f"fpm_match_staged_launch failed with {rc}: {self.last_error()}")

    def match_staged_finish_array(self):
        """Wait for the launched pass and post-process it (fpm_match_staged_finish); array views as
        match_staged_array.  On a full result buffer the results already computed are fetched into a larger one
        (fpm_last_results), without searching again."""
        n_src = self._staged
        _, out, n, views = self._views(n_src)
        rc = self._check(self._lib.fpm_match_staged_finish(self._ctx, out, self._cap, n), "match_staged_finish")
        if rc == L.FPM_E_CAPACITY:
            self._cap = max(self._cap * 2, max(n))
            _, out, n, views = self._views(n_src)
            rc = self._check(self._lib.fpm_last_results(self._ctx, out, self._cap, n), "last_results")
        if rc != L.FPM_OK:
            raise RuntimeError(f"fpm_match_staged_finish failed with {rc}: {self.last_error()}")
        return views

    # -- angle sharding of one search (fpm_set_angle_shard / fpm_last_candidates; sharding.match_angle_sharded) ----
    def setAngleShard(self, shard: int, shards: int):
        """Restrict searches to shard `shard` of `shards` contiguous blocks of the top-layer angle list."""
        rc = self._lib.fpm_set_angle_shard(self._ctx, int(shard), int(shards))
        if rc != L.FPM_OK:
            raise ValueError(f"fpm_set_angle_shard({shard}, {shards}) failed with {rc}: {self.last_error()}")

    def getAngleShard(self) -> Tuple[int, int]:
        a, b = C.c_int32(), C.c_int32()
        self._lib.fpm_get_angle_shard(self._ctx, C.byref(a), C.byref(b))
        return a.value, b.value

    def match_staged_candidates(self) -> List[np.ndarray]:
        """Search the staged sources and return each source's candidate records, skipping the host tail
        (fpm_match_staged_finish with out = NULL): the per-rank step of an angle-sharded search."""
        self.match_staged_launch()
        return self.match_staged_candidates_finish()

    def match_staged_candidates_finish(self) -> List[np.ndarray]:
        """Wait for a pass enqueued by match_staged_launch and return each source's candidate records (the second
        half of match_staged_candidates: a stream of passes over two contexts overlaps one's device pass with the
        other's record exchange and merge)."""
        n = (C.c_int32 * self._staged)()
        rc = self._check(self._lib.fpm_match_staged_finish(self._ctx, None, 0, n), "match_staged_finish")
        if rc != L.FPM_OK:
            raise RuntimeError(f"fpm_match_staged_finish failed with {rc}: {self.last_error()}")
        return [self.last_candidates(s) for s in range(self._staged)]

    def last_candidates_if_searched(self, source: int = 0):
        """last_candidates(source), or None when the last call ran no search for it (fpm_match returned before the
        device pass: empty source, unlearned template, size mismatch)."""
        n = C.c_int32()
        rc = self._lib.fpm_last_candidates(self._ctx, int(source), None, 0, C.byref(n))
        if rc not in (L.FPM_OK, L.FPM_E_CAPACITY):
            return None
        return self.last_candidates(source)

    def last_candidates(self, source: int = 0) -> np.ndarray:
        """Candidate records (CANDIDATE_DTYPE, push order) of `source` in the last search."""
        n = C.c_int32()
        rc = self._lib.fpm_last_candidates(self._ctx, int(source), None, 0, C.byref(n))
        if rc not in (L.FPM_OK, L.FPM_E_CAPACITY):
            raise ValueError(f"fpm_last_candidates({source}) failed with {rc}")
        out = np.zeros(n.value, CANDIDATE_DTYPE)
        if n.value:
            self._lib.fpm_last_candidates(self._ctx, int(source), out.ctypes.data_as(C.POINTER(L.Candidate)),
                                          n.value, C.byref(n))
        return out

    def search_bytes(self) -> Tuple[int, int, int]:
        """(B_pyr, B_top, B_ref): SURVEY.md §8(d) algorithmic bytes of the last search (fpm_search_bytes)."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        self._lib.fpm_search_bytes(self._ctx, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def search_stats(self) -> List[int]:
        buf = (C.c_int64 * 64)()
        k = self._lib.fpm_search_stats(self._ctx, buf, 64)
        return list(buf[:k])

    # -- setters / getters (TemplateMatcher.h:22-37) --------------------------------------------------------
    def resetParams(self):
        """Back to the reference constructor defaults (TemplateMatcher.cpp:28-39)."""
        self._lib.fpm_params_default(C.byref(self._params))

    def setMaxPositions(self, v: int): self._params.max_pos = int(v)
    def setMaxOverlap(self, v: float): self._params.max_overlap = float(v)
    def setScore(self, v: float): self._params.score = float(v)
    def setToleranceAngle(self, v: float): self._params.tolerance_angle = float(v)
    def setMinReduceArea(self, v: int): self._params.min_reduce_area = int(v)
    def setUseSIMD(self, v: bool): self._params.use_simd = 1 if v else 0
    def setSubPixelEstimation(self, v: bool): self._params.subpixel = 1 if v else 0
    def getMaxPositions(self) -> int: return self._params.max_pos
    def getMaxOverlap(self) -> float: return self._params.max_overlap
    def getScore(self) -> float: return self._params.score
    def getToleranceAngle(self) -> float: return self._params.tolerance_angle
    def getMinReduceArea(self) -> int: return self._params.min_reduce_area
    def getUseSIMD(self) -> bool: return bool(self._params.use_simd)
    def getSubPixelEstimation(self) -> bool: return bool(self._params.subpixel)
    def getLastExecutionTime(self) -> float: return self._last_time

    # -- user rectangle: stored only, unused by matching (TemplateMatcher.cpp:1224-1238) ---------------------
    def setUserDefinedRect(self, rect): self._user_rect = tuple(rect)
    def getUserDefinedRect(self): return self._user_rect if self._user_rect is not None else (0, 0, 0, 0)
    def hasUserDefinedRect(self) -> bool: return self._user_rect is not None

    # -- pixel operators (fpm_op_*) ---------------------------------------------------------------------------
    def pyr_down(self, img) -> np.ndarray:
        g = _gray(img)
        h, w = g.shape
        out = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
        rc = self._check(self._lib.fpm_op_pyr_down(self._ctx, L.u8ptr(g), w, h, g.strides[0], L.u8ptr(out),
                                                   out.strides[0]), "pyr_down")
        if rc != L.FPM_OK:
            raise ValueError(self.last_error())
        return out

    def pyr_down2(self, img, seg_chunks: int = 0, chunk_rows: int = 0):
        """(pyrDown(img), pyrDown(pyrDown(img))) from the search's two-level pyramid kernel (chunk_rows 16 / 32 forces
        its level-1 chunk height; 0 chooses it as the search does)."""
        g = _gray(img)
        h, w = g.shape
        b = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
        c = np.zeros(((b.shape[0] + 1) // 2, (b.shape[1] + 1) // 2), np.uint8)
        rc = self._check(self._lib.fpm_op_pyr_down2(self._ctx, L.u8ptr(g), w, h, g.strides[0], L.u8ptr(b), b.strides[0],
                                                    L.u8ptr(c), c.strides[0], int(seg_chunks), int(chunk_rows)),
                         "pyr_down2")
        if rc != L.FPM_OK:
            raise ValueError(self.last_error())
        return b, c

    def warp_affine(self, img, m, dsize, border: int = 0) -> np.ndarray:
        g = _gray(img)
        h, w = g.shape
        dw, dh = dsize
        out = np.zeros((dh, dw), np.uint8)
        mm = (C.c_double * 6)(*np.asarray(m, np.float64).ravel().tolist())
        rc = self._check(self._lib.fpm_op_warp_affine(self._ctx, L.u8ptr(g), w, h, g.strides[0], mm, L.u8ptr(out),
                                                      dw, dh, out.strides[0], int(border)), "warp_affine")
        if rc != L.FPM_OK:
            raise ValueError(self.last_error())
        return out

    def ncc_map(self, img, layer: int, fold: bool) -> np.ndarray:
        g = _gray(img)
        h, w = g.shape
        tw, th = self.template_level(layer)[0].shape[::-1]
        out = np.zeros((h - th + 1, w - tw + 1), np.float32)
        rc = self._check(self._lib.fpm_op_ncc_map(self._ctx, L.u8ptr(g), w, h, g.strides[0], int(layer),
                                                  1 if fold else 0,
                                                  out.ctypes.data_as(C.POINTER(C.c_float))), "ncc_map")
        if rc != L.FPM_OK:
            raise ValueError(self.last_error())
        return out

    def overlap_filter(self, corners, scores, max_overlap: float, device: bool = True):
        """filterWithRotatedRect (TemplateMatcher.cpp:1133-1194) on rectangles given as rows (ltx, lty, rtx, rty, rbx,
        rby) with their scores, in the given order: (indices of the survivors, stats) -- stats as fpm_op_overlap_filter
        (path, host-decided pairs, device fallback flags, pair entries)."""
        c = np.ascontiguousarray(corners, np.float32).reshape(-1, 6)
        sc = np.ascontiguousarray(scores, np.float64).ravel()
        n = c.shape[0]
        assert sc.shape[0] == n
        keep = np.zeros(max(n, 1), np.int32)
        st = np.zeros(4, np.int32)
        nk = C.c_int32()
        rc = self._lib.fpm_op_overlap_filter(self._ctx, c.ctypes.data_as(C.POINTER(C.c_float)),
                                             sc.ctypes.data_as(C.POINTER(C.c_double)), n, float(max_overlap),
                                             1 if device else 0, keep.ctypes.data_as(C.POINTER(C.c_int32)),
                                             C.byref(nk), st.ctypes.data_as(C.POINTER(C.c_int32)))
        if rc != L.FPM_OK:
            raise ValueError(self.last_error())
        return keep[:nk.value].tolist(), st.tolist()

    def template_info(self):
        lv, border = C.c_int32(), C.c_int32()
        rc = self._lib.fpm_template_info(self._ctx, C.byref(lv), C.byref(border))
        if rc != L.FPM_OK:
            raise ValueError("template not learned")
        return lv.value, border.value

    def template_level(self, level: int):
        w, h, eq = C.c_int32(), C.c_int32(), C.c_int32()
        mean, norm, inv = C.c_double(), C.c_double(), C.c_double()
        rc = self._lib.fpm_template_level(self._ctx, level, C.byref(w), C.byref(h), C.byref(mean), C.byref(norm),
                                          C.byref(inv), C.byref(eq), None, 0)
        if rc != L.FPM_OK:
            raise ValueError("bad level")
        px = np.zeros((h.value, w.value), np.uint8)
        self._lib.fpm_template_level(self._ctx, level, C.byref(w), C.byref(h), C.byref(mean), C.byref(norm),
                                     C.byref(inv), C.byref(eq), L.u8ptr(px), px.strides[0])
        return px, mean.value, norm.value, inv.value, bool(eq.value)

    # -- kernel timing ------------------------------------------------------------------------------------------
    def profile(self, enable: bool):
        self._lib.fpm_profile_enable(self._ctx, 1 if enable else 0)

    def profile_reset(self):
        self._lib.fpm_profile_reset(self._ctx)

    def profile_last(self):
        """(device_ms, host_ms, call_ms) of the last search call (fpm_profile_last)."""
        d, h, c = C.c_double(), C.c_double(), C.c_double()
        self._lib.fpm_profile_last(self._ctx, C.byref(d), C.byref(h), C.byref(c))
        return d.value, h.value, c.value

    def profile_get(self, kernel: int):
        ms, n, b = C.c_double(), C.c_int64(), C.c_int64()
        self._lib.fpm_profile_get(self._ctx, kernel, C.byref(ms), C.byref(n), C.byref(b))
        return ms.value, n.value, b.value
