"""ctypes view of libpsn_tracker2d.so (include/psn_tracker2d.h): the Tracker2D
flow stage -- backward feature-tracking chain, forward tracking + matching
score, LocalSearchKLT, PSN_Rect arithmetic -- of CPSNWhere_Tracker2D
(psn_where/PSNWhere_Tracker2D.cpp:452-1025) over the HIP LK library.

The records mirror the reference's stDetectedObject / stTracker2D fields that
the flow stage reads and writes. Everything calls the native library; there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

from ._lib import ERRORS

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSN_T2D_LIB") or os.path.join(_HERE, "lib", "libpsn_tracker2d.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "psn_tracker2d.h")

MAX_FEATURES = 100
MIN_FEATURES = 4
INTERVAL = 4
MAX_BOXES = 16
ERR_CAPACITY = -20


class T2dError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        name = "PSN_T2D_ERR_CAPACITY" if code == ERR_CAPACITY else ERRORS.get(code, code)
        super().__init__(f"{name}: {msg}")


class Rect(ctypes.Structure):
    _fields_ = [("x", ctypes.c_double), ("y", ctypes.c_double), ("w", ctypes.c_double), ("h", ctypes.c_double)]

    def tuple(self):
        return (self.x, self.y, self.w, self.h)


_PTS = ctypes.c_float * 2 * MAX_FEATURES


class Detection(ctypes.Structure):
    _fields_ = [
        ("box", Rect),
        ("num_features", ctypes.c_int),
        ("features", _PTS),
        ("valid", ctypes.c_int),
        ("overlap_other", ctypes.c_int),
        ("num_boxes", ctypes.c_int),
        ("boxes", Rect * INTERVAL),
        ("num_sets", ctypes.c_int),
        ("set_count", ctypes.c_int * INTERVAL),
        ("sets", _PTS * INTERVAL),
    ]


class Tracker(ctypes.Structure):
    _fields_ = [
        ("duration", ctypes.c_uint),
        ("num_boxes", ctypes.c_int),
        ("boxes", Rect * MAX_BOXES),
        ("num_features", ctypes.c_int),
        ("features", _PTS),
        ("num_tracked", ctypes.c_int),
        ("tracked", _PTS),
        ("updated", ctypes.c_int),
    ]


def header_functions() -> list[str]:
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(psn_\w+)\s*\(", src)))


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p
    dp = ctypes.POINTER(ctypes.c_double)
    L.psn_rect_overlap.argtypes = [Rect, Rect]
    L.psn_rect_distance.argtypes = [Rect, Rect]
    L.psn_rect_distance.restype = ctypes.c_double
    L.psn_rect_overlapped_area.argtypes = [Rect, Rect]
    L.psn_rect_overlapped_area.restype = ctypes.c_double
    L.psn_rect_contain.argtypes = [Rect, ctypes.c_float, ctypes.c_float]
    L.psn_rect_center.argtypes = [Rect, dp, dp]
    L.psn_rect_center.restype = None
    L.psn_t2d_box_matching_cost.argtypes = [Rect, Rect]
    L.psn_t2d_box_matching_cost.restype = ctypes.c_double
    L.psn_t2d_local_search_klt.argtypes = [Rect, fp, fp, ip, ctypes.POINTER(Rect), vp, ctypes.POINTER(ip)]
    L.psn_t2d_create.argtypes = [ip, ctypes.c_uint, ip, ip, ctypes.POINTER(vp)]
    L.psn_t2d_destroy.argtypes = [vp]
    L.psn_t2d_destroy.restype = None
    L.psn_t2d_last_error.argtypes = [vp]
    L.psn_t2d_last_error.restype = ctypes.c_char_p
    L.psn_t2d_push_frame.argtypes = [vp, vp, ip, ip]
    L.psn_t2d_rotate.argtypes = [vp]
    L.psn_t2d_detect_features.argtypes = [vp, ctypes.POINTER(Detection), ip, ctypes.c_uint32]
    L.psn_t2d_backward.argtypes = [vp, ctypes.POINTER(Detection), ip]
    L.psn_t2d_forward.argtypes = [vp, ctypes.POINTER(Tracker), ip, ctypes.POINTER(Detection), ip, fp]
    L.psn_t2d_track_frame.argtypes = [vp, ctypes.POINTER(Detection), ip, ctypes.POINTER(Tracker), ip, fp]
    _lib = L
    return L


def rect(x, y, w, h) -> Rect:
    return Rect(float(x), float(y), float(w), float(h))


def local_search_klt(pre_box, pre: np.ndarray, cur: np.ndarray):
    """LocalSearchKLT (PSNWhere_Tracker2D.cpp:455-554) -> (box tuple, inlier indices)."""
    pre = np.ascontiguousarray(pre, np.float32).reshape(-1, 2)
    cur = np.ascontiguousarray(cur, np.float32).reshape(-1, 2)
    n = len(pre)
    idx = np.zeros(max(n, 1), np.int32)
    out, ni = Rect(), ctypes.c_int()
    rc = load().psn_t2d_local_search_klt(rect(*pre_box), pre.ctypes.data, cur.ctypes.data, n, ctypes.byref(out),
                                         idx.ctypes.data, ctypes.byref(ni))
    if rc:
        raise T2dError(rc, "local_search_klt")
    return out.tuple(), idx[:ni.value].tolist()


def make_detection(box, features) -> Detection:
    d = Detection()
    d.box = rect(*box)
    f = np.asarray(features, np.float32).reshape(-1, 2)
    if len(f) > MAX_FEATURES:
        raise ValueError("more than PSN_T2D_MAX_FEATURES points")
    d.num_features = len(f)
    ctypes.memmove(d.features, f.ctypes.data, f.nbytes)
    return d


def make_tracker(boxes, features, duration=None) -> Tracker:
    t = Tracker()
    t.num_boxes = len(boxes)
    for i, b in enumerate(boxes):
        t.boxes[i] = rect(*b)
    t.duration = len(boxes) if duration is None else duration
    f = np.asarray(features, np.float32).reshape(-1, 2)
    t.num_features = len(f)
    ctypes.memmove(t.features, f.ctypes.data, f.nbytes)
    return t


def points(arr, n) -> np.ndarray:
    return np.ctypeslib.as_array(arr)[:n].copy()


class FlowTracker:
    """One camera's Tracker2D flow stage (psn_t2d)."""

    def __init__(self, width: int, height: int, cam_id: int = 0, device: int = 0):
        self._L = load()
        h = ctypes.c_void_p()
        rc = self._L.psn_t2d_create(device, cam_id, width, height, ctypes.byref(h))
        if rc:
            raise T2dError(rc, "psn_t2d_create")
        self._h = h
        self.width, self.height = width, height

    def _check(self, rc, what):
        if rc:
            raise T2dError(rc, f"{what}: {self._L.psn_t2d_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.psn_t2d_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def push_frame(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        ch = 1 if img.ndim == 2 else img.shape[2]
        self._check(self._L.psn_t2d_push_frame(self._h, img.ctypes.data, img.shape[1] * ch, ch), "push_frame")

    def rotate(self):
        self._check(self._L.psn_t2d_rotate(self._h), "rotate")

    def detect_features(self, dets: list[Detection], seed: int = 0):
        """GridFAST features of each detection on frame t (fills features / num_features)."""
        arr = (Detection * max(len(dets), 1))(*dets)
        self._check(self._L.psn_t2d_detect_features(self._h, arr, len(dets), ctypes.c_uint32(seed & 0xffffffff)),
                    "detect_features")
        return list(arr)[:len(dets)]

    def backward(self, dets: list[Detection]):
        arr = (Detection * max(len(dets), 1))(*dets)
        self._check(self._L.psn_t2d_backward(self._h, arr, len(dets)), "backward")
        return list(arr)[:len(dets)]

    def forward(self, trackers: list[Tracker], dets: list[Detection]):
        ta = (Tracker * max(len(trackers), 1))(*trackers)
        da = (Detection * max(len(dets), 1))(*dets)
        nvalid = sum(1 for d in dets if d.valid)
        cost = np.full(max(nvalid * len(trackers), 1), np.nan, np.float32)
        self._check(self._L.psn_t2d_forward(self._h, ta, len(trackers), da, len(dets), cost.ctypes.data), "forward")
        return list(ta)[:len(trackers)], cost[:nvalid * len(trackers)].reshape(nvalid, len(trackers))

    def track_frame(self, dets: list[Detection], trackers: list[Tracker]):
        da = (Detection * max(len(dets), 1))(*dets)
        ta = (Tracker * max(len(trackers), 1))(*trackers)
        cost = np.full(max(len(dets) * len(trackers), 1), np.nan, np.float32)
        self._check(self._L.psn_t2d_track_frame(self._h, da, len(dets), ta, len(trackers), cost.ctypes.data),
                    "track_frame")
        dets_out = list(da)[:len(dets)]
        nvalid = sum(1 for d in dets_out if d.valid)
        return dets_out, list(ta)[:len(trackers)], cost[:nvalid * len(trackers)].reshape(nvalid, len(trackers))
