"""Python view of the C ABI (include/psn_lk.h) for tests and bench.

`LKContext` is one camera's device ring of pyramids (the MI355X replacement of
CPSNWhere_Tracker2D's gray ring, PSNWhere_Tracker2D.cpp:256-263, :310-316) and
`calc_optical_flow_pyr_lk` mirrors cv::calcOpticalFlowPyrLK as called at
PSNWhere_Tracker2D.cpp:776-782 / :871-877: same argument meaning, same outputs
(nextPts written for every point, status, err), CV_Assert(winSize > 2)
surfaced as PsnLkError(PSN_LK_ERR_WINSIZE).

Everything here calls libpsn_lk.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import GridFastParams, LkParams, LkQuery, PsnLkError


def make_params(win_size=(21, 21), max_level=3, criteria=(3, 30, 0.01), flags=0,
                min_eig_threshold=1e-4) -> LkParams:
    p = LkParams()
    p.win_w, p.win_h = int(win_size[0]), int(win_size[1])
    p.max_level = int(max_level)
    p.term_type, p.max_count, p.epsilon = int(criteria[0]), int(criteria[1]), float(criteria[2])
    p.flags = int(flags)
    p.min_eig_threshold = float(min_eig_threshold)
    return p


def query_array(queries: list[LkQuery]):
    """The ctypes array psn_lk_track_device takes (at least one element; the
    number of real queries rides along as `nq`, 0 for an empty list)."""
    arr = (LkQuery * max(len(queries), 1))(*queries)
    arr.nq = len(queries)
    return arr


def make_query(prev_slot, next_slot, first_pt, num_pts, params: LkParams) -> LkQuery:
    q = LkQuery()
    q.prev_slot, q.next_slot, q.first_pt, q.num_pts = prev_slot, next_slot, first_pt, num_pts
    q.params = params
    return q


def gridfast_params(threshold=10, nonmax=True, max_total=1000, grid=(4, 4), cap=100) -> GridFastParams:
    """FeatureDetector::create("GridFAST") settings + the Tracker2D point cap."""
    p = GridFastParams()
    p.threshold, p.nonmax, p.max_total = int(threshold), int(bool(nonmax)), int(max_total)
    p.grid_rows, p.grid_cols, p.cap = int(grid[0]), int(grid[1]), int(cap)
    return p


def effective_max_level(width, height, win_w, win_h, max_level) -> int:
    return _lib.load().psn_lk_effective_max_level(width, height, win_w, win_h, max_level)


class LKContext:
    """One camera: device ring of `ring_slots` pyramids (max_level_cap+1 levels)."""

    def __init__(self, width: int, height: int, ring_slots: int = 4, max_level_cap: int = 3, device: int = 0,
                 variants: dict | None = None):
        self._L = _lib.load()
        self.width, self.height = width, height
        self.ring_slots, self.max_level_cap = ring_slots, max_level_cap
        h = ctypes.c_void_p()
        rc = self._L.psn_lk_create(device, width, height, ring_slots, max_level_cap, ctypes.byref(h))
        if rc != 0:
            raise PsnLkError(rc, "psn_lk_create")
        self._h = h
        for k, v in (variants or {}).items():
            self.set_variant(k, v)

    def set_variant(self, key: str, value: int):
        """Kernel-variant override (psn_lk_debug_set_variant): tests and experiments only."""
        self._check(self._L.psn_lk_debug_set_variant(self._h, _lib.VARIANTS[key], int(value)), f"set_variant {key}")

    def _check(self, rc, what):
        if rc != 0:
            raise PsnLkError(rc, f"{what}: {self._L.psn_lk_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.psn_lk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int | None):
        self._check(self._L.psn_lk_set_stream(self._h, stream_ptr), "set_stream")

    def set_ingest_overlap(self, mode=True):
        """Ingest overlap mode: False/0 off, True/1 internal ingest stream, 2 fused
        into the next LK launch's tail (see psn_lk_set_ingest_overlap)."""
        self._check(self._L.psn_lk_set_ingest_overlap(self._h, int(mode)), "set_ingest_overlap")

    def sync(self):
        self._check(self._L.psn_lk_sync(self._h), "sync")

    def push_frame(self, slot: int, img: np.ndarray):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        ch = 1 if img.ndim == 2 else img.shape[2]
        assert img.shape[0] == self.height and img.shape[1] == self.width
        self._check(self._L.psn_lk_push_frame(self._h, slot, img.ctypes.data, img.shape[1] * ch, ch), "push_frame")

    def push_frame_async(self, slot: int, img: np.ndarray):
        """Asynchronous upload + build (psn_lk_push_frame_async): `img` must stay
        alive and unchanged until sync() (pinned memory makes the copy async)."""
        ch = 1 if img.ndim == 2 else img.shape[2]
        assert img.flags["C_CONTIGUOUS"] and img.dtype == np.uint8
        self._check(self._L.psn_lk_push_frame_async(self._h, slot, img.ctypes.data, img.shape[1] * ch, ch),
                    "push_frame_async")

    def push_frame_jpeg(self, slot: int, data: bytes):
        """A baseline JPEG of the context's size, decoded on the device (psn_lk_push_frame_jpeg)."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._check(self._L.psn_lk_push_frame_jpeg(self._h, slot, buf, len(data)), "push_frame_jpeg")

    def push_frame_device(self, slot: int, dev_ptr: int, stride: int, channels: int = 1):
        self._check(self._L.psn_lk_push_frame_device(self._h, slot, dev_ptr, stride, channels), "push_frame_device")

    def read_level(self, slot: int, level: int) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.psn_lk_level_size(self._h, level, ctypes.byref(w), ctypes.byref(h)), "level_size")
        out = np.empty((h.value, w.value), np.uint8)
        self._check(self._L.psn_lk_read_level(self._h, slot, level, out.ctypes.data, w.value), "read_level")
        return out

    def track(self, queries: list[LkQuery], prev_pts: np.ndarray, next_pts: np.ndarray | None = None,
              want_err: bool = True):
        """Batched host-array LK. Returns (next_pts, status, err)."""
        prev = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(-1, 2)
        n = prev.shape[0]
        nxt = (np.zeros_like(prev) if next_pts is None
               else np.ascontiguousarray(next_pts, dtype=np.float32).reshape(-1, 2).copy())
        st = np.zeros(n, np.uint8)
        er = np.zeros(n, np.float32) if want_err else None
        arr = (LkQuery * max(len(queries), 1))(*queries)
        self._check(self._L.psn_lk_track(self._h, arr, len(queries), prev.ctypes.data, nxt.ctypes.data,
                                         st.ctypes.data, er.ctypes.data if er is not None else None), "track")
        return nxt, st, er

    def track_device(self, queries, d_prev: int, d_next: int, d_status: int, d_err: int | None):
        """`queries`: a list of LkQuery, or a ctypes LkQuery array built once by the
        caller (query_array) for a launch it repeats."""
        arr = queries if isinstance(queries, ctypes.Array) else query_array(queries)
        nq = getattr(arr, "nq", len(arr))
        self._check(self._L.psn_lk_track_device(self._h, arr, nq, d_prev, d_next, d_status, d_err), "track_device")

    def gridfast_detect(self, slot: int, rois, params: GridFastParams | None = None, seed: int = 0):
        """GridFAST keypoints of slot's frame masked by each roi (x, y, w, h),
        shuffled by `seed` and capped (PSNWhere_Tracker2D.cpp:734-757).
        Returns (list of (n_i, 2) f32 point arrays, totals before the cap)."""
        p = params or gridfast_params()
        r = np.ascontiguousarray(np.asarray(rois, dtype=np.int32).reshape(-1, 4))
        n = r.shape[0]
        cap = max(p.cap, 0)
        xy = np.zeros((max(n, 1), max(cap, 1), 2), np.float32)
        cnt = np.zeros(max(n, 1), np.int32)
        tot = np.zeros(max(n, 1), np.int32)
        self._check(self._L.psn_gridfast_detect(self._h, slot, r.ctypes.data, n, ctypes.byref(p),
                                                ctypes.c_uint32(seed & 0xffffffff), xy.ctypes.data,
                                                cnt.ctypes.data, tot.ctypes.data), "gridfast_detect")
        return [xy[i, :cnt[i]].copy() for i in range(n)], tot[:n].copy()

    def gridfast_detect_device(self, slot: int, rois, params: GridFastParams | None, seed: int, d_xy: int,
                               d_count: int, d_total: int | None):
        p = params or gridfast_params()
        r = np.ascontiguousarray(np.asarray(rois, dtype=np.int32).reshape(-1, 4))
        self._check(self._L.psn_gridfast_detect_device(self._h, slot, r.ctypes.data, r.shape[0], ctypes.byref(p),
                                                       ctypes.c_uint32(seed & 0xffffffff), d_xy, d_count, d_total),
                    "gridfast_detect_device")

    def gridfast_detect_sets(self, slots, roi_sets, params: GridFastParams | None = None, seed: int = 0):
        """psn_gridfast_detect_device_sets: set i = roi_sets[i] on ring slot
        slots[i], all sets in as few launches as possible. Returns, per set,
        (list of (n_j, 2) f32 point arrays, totals before the cap) -- what
        gridfast_detect(slots[i], roi_sets[i]) returns."""
        from . import hip

        p = params or gridfast_params()
        sets = [np.asarray(r, dtype=np.int32).reshape(-1, 4) for r in roi_sets]
        nrois = np.array([r.shape[0] for r in sets], np.int32)
        sl = np.ascontiguousarray(np.asarray(slots, np.int32))
        if sl.shape[0] != len(sets):
            raise ValueError("one slot per roi set")
        r = np.ascontiguousarray(np.concatenate(sets + [np.zeros((0, 4), np.int32)]))
        n, cap = r.shape[0], max(p.cap, 0)
        d_xy = hip.DeviceBuffer(max(n, 1) * max(cap, 1) * 8)
        d_cnt, d_tot = hip.DeviceBuffer(max(n, 1) * 4), hip.DeviceBuffer(max(n, 1) * 4)
        try:
            self._check(self._L.psn_gridfast_detect_device_sets(
                self._h, len(sets), sl.ctypes.data, nrois.ctypes.data, r.ctypes.data, ctypes.byref(p),
                ctypes.c_uint32(seed & 0xffffffff), d_xy.addr, d_cnt.addr, d_tot.addr), "gridfast_detect_sets")
            xy = d_xy.to_array((max(n, 1), max(cap, 1), 2), np.float32)
            cnt = d_cnt.to_array(max(n, 1), np.int32)
            tot = d_tot.to_array(max(n, 1), np.int32)
        finally:
            for b in (d_xy, d_cnt, d_tot):
                b.free()
        out, k = [], 0
        for m in nrois:
            out.append(([xy[k + j, :cnt[k + j]].copy() for j in range(m)], tot[k:k + m].copy()))
            k += m
        return out

    def track_device_counted(self, queries: list[LkQuery], d_counts: int, d_prev: int, d_next: int, d_status: int,
                             d_err: int | None):
        """Queries sized num_pts (capacity); query i processes d_counts[i] points (device int32)."""
        arr = (LkQuery * max(len(queries), 1))(*queries)
        self._check(self._L.psn_lk_track_device_counted(self._h, arr, len(queries), d_counts, d_prev, d_next,
                                                        d_status, d_err), "track_device_counted")

    def track_device_counted_strided(self, queries: list[LkQuery], d_counts: int, count_stride: int, d_prev: int,
                                     d_next: int, d_status: int, d_err: int | None):
        """As track_device_counted with query i's count at d_counts[i * count_stride]."""
        arr = (LkQuery * max(len(queries), 1))(*queries)
        self._check(self._L.psn_lk_track_device_counted_strided(self._h, arr, len(queries), d_counts, count_stride,
                                                                d_prev, d_next, d_status, d_err),
                    "track_device_counted_strided")

    def enable_timing(self, capacity: int = 1024, every: int = 1):
        """HIP-event timing of every `every`-th push (pyramid launch) / track (LK launch) call."""
        self._check(self._L.psn_lk_enable_timing(self._h, int(capacity), int(every)), "enable_timing")

    def timing_stats(self) -> dict:
        np_, nt = ctypes.c_int(), ctypes.c_int()
        pm, tm = ctypes.c_double(), ctypes.c_double()
        self._check(self._L.psn_lk_timing_stats(self._h, ctypes.byref(np_), ctypes.byref(pm), ctypes.byref(nt),
                                                ctypes.byref(tm)), "timing_stats")
        return {"n_push": np_.value, "push_ms": pm.value, "n_track": nt.value, "track_ms": tm.value}

    def calc_optical_flow_pyr_lk(self, prev_img, next_img, prev_pts, win_size=(21, 21), max_level=3,
                                 criteria=(3, 30, 0.01), flags=0, min_eig_threshold=1e-4, next_pts=None,
                                 want_err=True):
        prev_img = np.ascontiguousarray(prev_img, dtype=np.uint8)
        next_img = np.ascontiguousarray(next_img, dtype=np.uint8)
        pts = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(-1, 2)
        n = pts.shape[0]
        nxt = (np.zeros_like(pts) if next_pts is None
               else np.ascontiguousarray(next_pts, dtype=np.float32).reshape(-1, 2).copy())
        st = np.zeros(n, np.uint8)
        er = np.zeros(n, np.float32) if want_err else None
        p = make_params(win_size, max_level, criteria, flags, min_eig_threshold)
        self._check(self._L.psn_calc_optical_flow_pyr_lk(
            self._h, prev_img.ctypes.data, next_img.ctypes.data, prev_img.shape[1], pts.ctypes.data,
            nxt.ctypes.data, st.ctypes.data, er.ctypes.data if er is not None else None, n, ctypes.byref(p)),
            "calc_optical_flow_pyr_lk")
        return nxt, st, er


def calc_optical_flow_pyr_lk(prev_img, next_img, prev_pts, win_size=(21, 21), max_level=3,
                             criteria=(3, 30, 0.01), flags=0, min_eig_threshold=1e-4, next_pts=None,
                             want_err=True, device=0, variants=None):
    """cv::calcOpticalFlowPyrLK on MI355X (one-shot; allocates a context).
    `variants`: kernel-variant overrides for tests (LKContext.set_variant)."""
    h, w = np.asarray(prev_img).shape[:2]
    cap = max(0, effective_max_level(w, h, win_size[0], win_size[1], max_level))
    with LKContext(w, h, ring_slots=1, max_level_cap=min(cap, 5), device=device, variants=variants) as ctx:
        return ctx.calc_optical_flow_pyr_lk(prev_img, next_img, prev_pts, win_size, max_level, criteria,
                                            flags, min_eig_threshold, next_pts, want_err)


class SGSmoother:
    """Batched CPSNWhere_SGSmooth (psn_sgsmooth.h): `nseries` trajectories of
    `dims` coordinates, one Insert per series per call, on the device."""

    def __init__(self, nseries: int, dims: int = 2, span: int = 9, degree: int = 1, device: int = 0):
        self._L = _lib.load()
        self.nseries, self.dims, self.span = nseries, dims, span
        h = ctypes.c_void_p()
        rc = self._L.psn_sg_create(device, nseries, dims, span, degree, ctypes.byref(h))
        if rc != 0:
            raise PsnLkError(rc, "psn_sg_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.psn_sg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert(self, values: np.ndarray, active: np.ndarray | None = None):
        """values (nseries, >= dims) f32. Returns (refresh (n,) int32, out (n, span, dims) f64):
        row k of series i = smoothed position refresh[i] + k (rows < length - refresh valid)."""
        v = np.ascontiguousarray(values, dtype=np.float32).reshape(self.nseries, -1)
        act = None if active is None else np.ascontiguousarray(active, dtype=np.uint8)
        ref = np.zeros(self.nseries, np.int32)
        out = np.zeros((self.nseries, self.span, self.dims), np.float64)
        rc = self._L.psn_sg_insert(self._h, v.ctypes.data, v.shape[1], act.ctypes.data if act is not None else None,
                                   ref.ctypes.data, out.ctypes.data)
        if rc != 0:
            raise PsnLkError(rc, "psn_sg_insert")
        return ref, out

    def set_stream(self, stream_ptr: int | None):
        rc = self._L.psn_sg_set_stream(self._h, stream_ptr)
        if rc != 0:
            raise PsnLkError(rc, "psn_sg_set_stream")

    def insert_device(self, d_in: int, in_stride: int, d_active: int | None, d_refresh: int, d_out: int):
        rc = self._L.psn_sg_insert_device(self._h, d_in, in_stride, d_active, d_refresh, d_out)
        if rc != 0:
            raise PsnLkError(rc, "psn_sg_insert_device")

    def lengths(self) -> np.ndarray:
        n = np.zeros(self.nseries, np.int32)
        rc = self._L.psn_sg_lengths(self._h, n.ctypes.data)
        if rc != 0:
            raise PsnLkError(rc, "psn_sg_lengths")
        return n


class JpegDecoder:
    """psn_jpeg (include/psn_jpeg.h): baseline JPEG -> BGR on the device."""

    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        rc = self._L.psn_jpeg_create(device, ctypes.byref(h))
        if rc != 0:
            raise PsnLkError(rc, "psn_jpeg_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.psn_jpeg_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def info(data: bytes):
        w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = _lib.load().psn_jpeg_info(data, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c))
        if rc != 0:
            raise PsnLkError(rc, "psn_jpeg_info")
        return w.value, h.value, c.value

    def decode(self, data: bytes) -> np.ndarray:
        """(H, W, 3) u8 BGR, as cv::imread(..., IMREAD_COLOR) returns it."""
        w, h, _ = self.info(data)
        out = np.empty((h, w, 3), np.uint8)
        rc = self._L.psn_jpeg_decode(self._h, data, len(data), out.ctypes.data, 3 * w)
        if rc != 0:
            raise PsnLkError(rc, f"psn_jpeg_decode: {self._L.psn_jpeg_last_error(self._h).decode()}")
        return out
