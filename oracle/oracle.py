"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/liblk_oracle.so, the CPU restatement of the
OpenCV 2.4.6 pyramidal-LK path behind CPSNWhere_Tracker2D
(psn_where/PSNWhere_Tracker2D.cpp:776-782, :871-877). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product path (mcmtt_opticalflow_amd) never does.

PARITY UNPINNED: OpenCV 2.4.6 (the pinned dependency, psn_where/PSN_Where.vcxproj:
97,104,124-125,151,175-176) is absent here and the reference holds no fixtures.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblk_oracle.so")
_lib = None

ACCUM_SSE2 = 0
ACCUM_SCALAR = 1
ACCUM_EXACT = 2  # analysis only: order-free int64 window sums (lk_oracle.h ORACLE_ACCUM_EXACT)
USE_INITIAL_FLOW = 4
GET_MIN_EIGENVALS = 8

_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_i16p = ctypes.POINTER(ctypes.c_int16)


def build() -> str:
    """Compile liblk_oracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_refl101.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_refl101.restype = ctypes.c_int
        L.oracle_bgr2gray.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, ctypes.c_int]
        L.oracle_pyr_down.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, ctypes.c_int]
        L.oracle_scharr.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i16p, ctypes.c_int]
        L.oracle_effective_max_level.argtypes = [ctypes.c_int] * 5
        L.oracle_effective_max_level.restype = ctypes.c_int
        L.oracle_level_offset.argtypes = [ctypes.c_int] * 3
        L.oracle_level_offset.restype = ctypes.c_long
        L.oracle_build_pyramid.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        common = [_f32p, _f32p, _u8p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_double,
                  ctypes.c_int, ctypes.c_int]
        L.oracle_lk_track_pyr.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int] + common
        L.oracle_lk_track_pyr.restype = ctypes.c_int
        L.oracle_calc_optical_flow_pyr_lk.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + common
        L.oracle_calc_optical_flow_pyr_lk.restype = ctypes.c_int
        ip = ctypes.c_int
        _i32p = ctypes.POINTER(ctypes.c_int)
        L.oracle_fast16.argtypes = [_u8p, ip, ip, ip, ip, ip, _i32p, _i32p, _i32p, ip]
        L.oracle_fast16.restype = ip
        L.oracle_gridfast.argtypes = [_u8p, ip, ip, ip, ip, ip, ip, ip, ip, ip, ip, ip, ip, _f32p, _i32p, ip]
        L.oracle_gridfast.restype = ip
        L.oracle_gridfast_key.argtypes = [ctypes.c_uint32] * 3
        L.oracle_gridfast_key.restype = ctypes.c_uint32
        L.oracle_gridfast_select.argtypes = [_f32p, ip, ctypes.c_uint32, ip, ip, _f32p]
        L.oracle_gridfast_select.restype = ip
        L.oracle_jpeg_info.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _i32p, _i32p, _i32p]
        L.oracle_jpeg_decode_bgr.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _u8p, ip]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def refl101(p: int, n: int) -> int:
    return lib().oracle_refl101(p, n)


def bgr2gray(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w, _ = img.shape
    out = np.empty((h, w), np.uint8)
    lib().oracle_bgr2gray(_p(img, _u8p), w, h, w * 3, _p(out, _u8p), w)
    return out


def pyr_down(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.empty(((h + 1) // 2, (w + 1) // 2), np.uint8)
    lib().oracle_pyr_down(_p(img, _u8p), w, h, w, _p(out, _u8p), out.shape[1])
    return out


def scharr(img: np.ndarray) -> np.ndarray:
    """Returns int16 array (h, w, 2) = (Ix, Iy)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.empty((h, w, 2), np.int16)
    lib().oracle_scharr(_p(img, _u8p), w, h, w, _p(out, _i16p), 2 * w)
    return out


def effective_max_level(w, h, win_w, win_h, max_level) -> int:
    return lib().oracle_effective_max_level(w, h, win_w, win_h, max_level)


def build_pyramid(img: np.ndarray, nlevels: int) -> list[np.ndarray]:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    total = lib().oracle_level_offset(w, h, nlevels)
    buf = np.empty(total, np.uint8)
    lib().oracle_build_pyramid(_p(img, _u8p), w, h, w, nlevels, _p(buf, _u8p))
    out = []
    lw, lh, off = w, h, 0
    for _ in range(nlevels):
        out.append(buf[off:off + lw * lh].reshape(lh, lw).copy())
        off += lw * lh
        lw, lh = (lw + 1) // 2, (lh + 1) // 2
    return out


def build_pyramid_packed(img: np.ndarray, nlevels: int) -> np.ndarray:
    """The packed pyramid buffer lk_track_pyr takes (levels back to back)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    buf = np.empty(lib().oracle_level_offset(w, h, nlevels), np.uint8)
    lib().oracle_build_pyramid(_p(img, _u8p), w, h, w, nlevels, _p(buf, _u8p))
    return buf


def lk_track_pyr(prev_pyr, next_pyr, w, h, prev_pts, win_size, max_level, criteria=(3, 30, 0.01), flags=0,
                 min_eig_threshold=1e-4, accum=ACCUM_SSE2, nthreads=0, want_err=True):
    """LK over prebuilt packed pyramids (the shared-pyramid schedule); max_level
    is truncated here as buildOpticalFlowPyramid would."""
    pts = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(-1, 2)
    n = pts.shape[0]
    nxt = np.zeros_like(pts)
    st = np.zeros(n, np.uint8)
    er = np.zeros(n, np.float32) if want_err else None
    ml = effective_max_level(w, h, win_size[0], win_size[1], max_level)
    rc = lib().oracle_lk_track_pyr(_p(prev_pyr, _u8p), _p(next_pyr, _u8p), w, h, _p(pts, _f32p), _p(nxt, _f32p),
                                   _p(st, _u8p), _p(er, _f32p) if er is not None else None, n, win_size[0],
                                   win_size[1], ml, criteria[0], criteria[1], criteria[2], flags, min_eig_threshold,
                                   accum, nthreads)
    if rc != 0:
        raise ValueError(f"oracle_lk_track_pyr failed rc={rc}")
    return nxt, st, er


def calc_optical_flow_pyr_lk(prev_img, next_img, prev_pts, win_size=(21, 21), max_level=3,
                             criteria=(3, 30, 0.01), flags=0, min_eig_threshold=1e-4,
                             next_pts=None, accum=ACCUM_SSE2, nthreads=0, want_err=True):
    """cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts, status, err, winSize,
    maxLevel, criteria, flags, minEigThreshold) with the reference call schedule
    (both pyramids rebuilt inside). Returns (next_pts (n,2) f32, status (n,) u8,
    err (n,) f32 or None)."""
    prev_img = np.ascontiguousarray(prev_img, dtype=np.uint8)
    next_img = np.ascontiguousarray(next_img, dtype=np.uint8)
    h, w = prev_img.shape
    pts = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(-1, 2)
    n = pts.shape[0]
    nxt = (np.zeros_like(pts) if next_pts is None
           else np.ascontiguousarray(next_pts, dtype=np.float32).reshape(-1, 2).copy())
    st = np.zeros(n, np.uint8)
    er = np.zeros(n, np.float32) if want_err else None
    rc = lib().oracle_calc_optical_flow_pyr_lk(
        _p(prev_img, _u8p), _p(next_img, _u8p), w, h, w, _p(pts, _f32p), _p(nxt, _f32p),
        _p(st, _u8p), _p(er, _f32p) if er is not None else None, n, win_size[0], win_size[1],
        max_level, criteria[0], criteria[1], criteria[2], flags, min_eig_threshold, accum, nthreads)
    if rc != 0:
        raise ValueError(f"oracle_calc_optical_flow_pyr_lk failed rc={rc}")
    return nxt, st, er


# ---- GridFAST (oracle/gridfast_oracle.c) ----

def fast16(img, threshold=10, nonmax=True):
    """FAST_t<16> of OpenCV 2.4.6 on a whole image: (n, 3) int32 rows (x, y, response)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = w * h
    kx, ky, kr = (np.empty(max(cap, 1), np.int32) for _ in range(3))
    ip = ctypes.POINTER(ctypes.c_int)
    n = lib().oracle_fast16(_p(img, _u8p), w, h, w, threshold, int(nonmax), _p(kx, ip), _p(ky, ip), _p(kr, ip), cap)
    return np.stack([kx[:n], ky[:n], kr[:n]], axis=1)


def gridfast(img, roi, threshold=10, nonmax=True, max_total=1000, grid=(4, 4)):
    """GridAdaptedFeatureDetector(FAST)::detect(img, kps, mask = 255 on roi):
    ((n, 2) f32 points in cell order, (n,) int32 responses)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = max(max_total, 1)
    xy = np.empty((cap, 2), np.float32)
    resp = np.empty(cap, np.int32)
    n = lib().oracle_gridfast(_p(img, _u8p), w, h, w, int(roi[0]), int(roi[1]), int(roi[2]), int(roi[3]),
                              threshold, int(nonmax), max_total, grid[0], grid[1], _p(xy, _f32p),
                              _p(resp, ctypes.POINTER(ctypes.c_int)), cap)
    return xy[:n].copy(), resp[:n].copy()


def gridfast_select(cand_xy, seed, roi_index, cap=100):
    """The seeded shuffle + cap (definition shared with the HIP kernel)."""
    c = np.ascontiguousarray(cand_xy, dtype=np.float32).reshape(-1, 2)
    out = np.empty((max(min(len(c), cap), 1), 2), np.float32)
    m = lib().oracle_gridfast_select(_p(c, _f32p), len(c), seed & 0xffffffff, roi_index, cap, _p(out, _f32p))
    return out[:m].copy()


def gridfast_detect(img, rois, seed=0, threshold=10, nonmax=True, max_total=1000, grid=(4, 4), cap=100):
    """Per roi: (points after shuffle + cap, total keypoints) -- what
    psn_gridfast_detect returns."""
    pts, tots = [], []
    for i, r in enumerate(rois):
        xy, _ = gridfast(img, r, threshold, nonmax, max_total, grid)
        pts.append(gridfast_select(xy, seed, i, cap))
        tots.append(len(xy))
    return pts, np.asarray(tots, np.int32)


# ---- JPEG decode (oracle/jpeg_oracle.c) ----

def jpeg_decode_bgr(data: bytes) -> np.ndarray:
    """cv::imread(..., IMREAD_COLOR) of a baseline JPEG: (H, W, 3) u8 BGR."""
    buf = np.frombuffer(data, np.uint8)
    w, h, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if lib().oracle_jpeg_info(buf.ctypes.data, buf.size, ctypes.byref(w), ctypes.byref(h), ctypes.byref(nc)) != 0:
        raise ValueError("not a baseline JPEG")
    out = np.zeros((h.value, w.value, 3), np.uint8)
    rc = lib().oracle_jpeg_decode_bgr(buf.ctypes.data, buf.size, _p(out, _u8p), 3 * w.value)
    if rc != 0:
        raise ValueError(f"oracle_jpeg_decode_bgr failed rc={rc}")
    return out
