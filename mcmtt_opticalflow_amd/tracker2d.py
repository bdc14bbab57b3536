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
LIB_PATH = os.path.join(_HERE, "lib", "libpsn_tracker2d.so")
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
        ("head", Rect),
        ("location", ctypes.c_double * 3),
        ("height", ctypes.c_double),
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
        ("id", ctypes.c_uint),
        ("time_start", ctypes.c_uint),
        ("time_end", ctypes.c_uint),
        ("time_last_update", ctypes.c_uint),
        ("duration", ctypes.c_uint),
        ("num_boxes", ctypes.c_int),
        ("boxes", Rect * MAX_BOXES),
        ("heads", Rect * MAX_BOXES),
        ("last_position", ctypes.c_double * 3),
        ("height", ctypes.c_double),
        ("confidence", ctypes.c_double),
        ("num_features", ctypes.c_int),
        ("features", _PTS),
        ("num_tracked", ctypes.c_int),
        ("tracked", _PTS),
        ("updated", ctypes.c_int),
    ]


class Object2D(ctypes.Structure):  # psn_object2d (stObject2DInfo)
    _fields_ = [("id", ctypes.c_uint), ("box", Rect), ("head", Rect), ("score", ctypes.c_double),
                ("num_prev", ctypes.c_int), ("prev", (ctypes.c_float * 2) * MAX_FEATURES),
                ("num_curr", ctypes.c_int), ("curr", (ctypes.c_float * 2) * MAX_FEATURES)]


class Track2DResult(ctypes.Structure):  # psn_track2d_result (stTrack2DResult)
    _fields_ = [("cam_id", ctypes.c_uint), ("frame_idx", ctypes.c_uint),
                ("num_objects", ctypes.c_int), ("cap_objects", ctypes.c_int), ("objects", ctypes.POINTER(Object2D)),
                ("num_detection_rects", ctypes.c_int), ("cap_detection_rects", ctypes.c_int),
                ("detection_rects", ctypes.POINTER(Rect)),
                ("num_tracker_rects", ctypes.c_int), ("cap_tracker_rects", ctypes.c_int),
                ("tracker_rects", ctypes.POINTER(Rect))]


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
    L.psn_t2d_push_frame_device.argtypes = [vp, vp, ip, ip]
    L.psn_t2d_track_frame_detect.argtypes = [vp, vp, ip, ctypes.c_uint32, vp, ip, vp]
    L.psn_t2d_lk_context.argtypes = [vp]
    L.psn_t2d_lk_context.restype = vp
    L.psn_t2d_rotate.argtypes = [vp]
    L.psn_t2d_write_result_txt.argtypes = [ctypes.c_char_p, ctypes.POINTER(Track2DResult)]
    L.psn_t2d_read_result_txt.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(Track2DResult)]
    L.psn_t2d_result_slot_bytes.argtypes = [ip, ip]
    L.psn_t2d_result_slot_bytes.restype = ctypes.c_size_t
    L.psn_t2d_pack_result.argtypes = [ctypes.POINTER(Track2DResult), vp, ctypes.c_size_t]
    L.psn_t2d_unpack_result.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(Track2DResult)]
    L.psn_t2d_set_device_chain.argtypes = [vp, ip]
    L.psn_t2d_detect_features.argtypes = [vp, ctypes.POINTER(Detection), ip, ctypes.c_uint32]
    L.psn_t2d_backward.argtypes = [vp, ctypes.POINTER(Detection), ip]
    L.psn_t2d_forward.argtypes = [vp, ctypes.POINTER(Tracker), ip, ctypes.POINTER(Detection), ip, fp]
    L.psn_t2d_track_frame.argtypes = [vp, ctypes.POINTER(Detection), ip, ctypes.POINTER(Tracker), ip, fp]
    L.psn_t2d_abi_version.restype = ip
    L.psn_t2d_assign.argtypes = [fp, ip, ip, vp]
    L.psn_t2d_hungarian_match.argtypes = [fp, ip, ip, vp, vp, fp, ctypes.POINTER(ip)]
    L.psn_t2d_result_with_tracker.argtypes = [ctypes.POINTER(Tracker), ctypes.POINTER(Object2D)]
    L.psn_t2d_matching_and_updating.argtypes = [ctypes.POINTER(Detection), ip, ctypes.POINTER(Tracker), ip, fp, vp,
                                                ctypes.c_uint, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(Tracker),
                                                ip, ctypes.POINTER(ip), ctypes.POINTER(Track2DResult)]
    L.psn_t2d_group_create.argtypes = [ip, ip, vp, ip, ip, ctypes.POINTER(vp)]
    L.psn_t2d_group_destroy.argtypes = [vp]
    L.psn_t2d_group_destroy.restype = None
    L.psn_t2d_group_last_error.argtypes = [vp]
    L.psn_t2d_group_last_error.restype = ctypes.c_char_p
    L.psn_t2d_group_lk_context.argtypes = [vp]
    L.psn_t2d_group_lk_context.restype = vp
    L.psn_t2d_group_push_frame.argtypes = [vp, ip, vp, ip, ip]
    L.psn_t2d_group_push_frame_device.argtypes = [vp, ip, vp, ip, ip]
    L.psn_t2d_group_push_frame_jpeg.argtypes = [vp, ip, vp, ctypes.c_size_t]
    L.psn_t2d_group_launch.argtypes = [vp, ctypes.c_uint, vp, vp, ip, ctypes.c_uint32]
    L.psn_t2d_group_complete.argtypes = [vp, vp, vp, ctypes.POINTER(Track2DResult)]
    L.psn_t2d_group_run.argtypes = [vp, ctypes.c_uint, vp, vp, ip, ctypes.c_uint32, ctypes.POINTER(Track2DResult)]
    L.psn_t2d_group_complete_next.argtypes = [vp, vp, vp, ctypes.POINTER(Track2DResult), ctypes.c_uint, vp, vp, ip,
                                              ctypes.c_uint32]
    L.psn_t2d_group_trackers.argtypes = [vp, ip, ctypes.POINTER(Tracker), ip, ctypes.POINTER(ip)]
    L.psn_t2d_group_debug_host_times.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.psn_t2d_group_debug_host_match_times.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
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


def make_detection(box, features, head=None, location=(0.0, 0.0, 0.0), height=0.0) -> Detection:
    """A detection record: box, features at t, head box (vecPartBoxes.front(); default: the box)
    and the caller's 3D estimate (location, height)."""
    d = Detection()
    d.box = rect(*box)
    d.head = rect(*(head if head is not None else box))
    for k in range(3):
        d.location[k] = float(location[k])
    d.height = float(height)
    f = np.asarray(features, np.float32).reshape(-1, 2)
    if len(f) > MAX_FEATURES:
        raise ValueError("more than PSN_T2D_MAX_FEATURES points")
    d.num_features = len(f)
    ctypes.memmove(d.features, f.ctypes.data, f.nbytes)
    return d


def make_tracker(boxes, features, duration=None, heads=None, id_=0) -> Tracker:
    t = Tracker()
    t.id = id_
    t.num_boxes = len(boxes)
    for i, b in enumerate(boxes):
        t.boxes[i] = rect(*b)
        t.heads[i] = rect(*(heads[i] if heads is not None else b))
    t.duration = len(boxes) if duration is None else duration
    t.confidence = 1.0
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

    def set_device_chain(self, on: bool):
        """LocalSearchKLT chain steps on the device (default) or on the host."""
        self._check(self._L.psn_t2d_set_device_chain(self._h, int(bool(on))), "set_device_chain")

    def push_frame(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        ch = 1 if img.ndim == 2 else img.shape[2]
        self._check(self._L.psn_t2d_push_frame(self._h, img.ctypes.data, img.shape[1] * ch, ch), "push_frame")

    def push_frame_device(self, dev_ptr: int, stride: int, channels: int = 1):
        """Ingest a frame already in device memory (e.g. a torch tensor's data_ptr())."""
        self._check(self._L.psn_t2d_push_frame_device(self._h, ctypes.c_void_p(dev_ptr), stride, channels),
                    "push_frame_device")

    def lk_handle(self) -> int:
        """The flow stage's psn_lk_ctx (kernel timing, stream)."""
        return self._L.psn_t2d_lk_context(self._h)

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

    def track_frame_detect(self, dets: list[Detection], trackers: list[Tracker], seed: int = 0):
        """detect_features + track_frame in one device pass (psn_t2d_track_frame_detect)."""
        da = (Detection * max(len(dets), 1))(*dets)
        ta = (Tracker * max(len(trackers), 1))(*trackers)
        cost = np.full(max(len(dets) * len(trackers), 1), np.nan, np.float32)
        self._check(self._L.psn_t2d_track_frame_detect(self._h, da, len(dets), seed & 0xffffffff, ta, len(trackers),
                                                       cost.ctypes.data), "track_frame_detect")
        dets_out = list(da)[:len(dets)]
        nvalid = sum(1 for d in dets_out if d.valid)
        return dets_out, list(ta)[:len(trackers)], cost[:nvalid * len(trackers)].reshape(nvalid, len(trackers))

    def track_frame(self, dets: list[Detection], trackers: list[Tracker]):
        da = (Detection * max(len(dets), 1))(*dets)
        ta = (Tracker * max(len(trackers), 1))(*trackers)
        cost = np.full(max(len(dets) * len(trackers), 1), np.nan, np.float32)
        self._check(self._L.psn_t2d_track_frame(self._h, da, len(dets), ta, len(trackers), cost.ctypes.data),
                    "track_frame")
        dets_out = list(da)[:len(dets)]
        nvalid = sum(1 for d in dets_out if d.valid)
        return dets_out, list(ta)[:len(trackers)], cost[:nvalid * len(trackers)].reshape(nvalid, len(trackers))


def assign(cost: np.ndarray) -> list[int]:
    """psn_t2d_assign: the Hungarian step of Track2D_MatchingAndUpdating -> column per row or -1."""
    c = np.ascontiguousarray(cost, np.float32)
    rows, cols = c.shape
    m = np.full(max(rows, 1), -2, np.int32)
    rc = load().psn_t2d_assign(c.ctypes.data, rows, cols, m.ctypes.data)
    if rc:
        raise T2dError(rc, "psn_t2d_assign")
    return m[:rows].tolist()


def hungarian_match(cost: np.ndarray):
    """psn_t2d_hungarian_match (CPSNWhere_Hungarian::Match) -> (rows, cols, costs) of the matched pairs."""
    c = np.ascontiguousarray(cost, np.float32)
    rows, cols = c.shape
    cap = max(min(rows, cols), 1)
    r, k, v = np.zeros(cap, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.float32)
    n = ctypes.c_int()
    rc = load().psn_t2d_hungarian_match(c.ctypes.data, rows, cols, r.ctypes.data, k.ctypes.data, v.ctypes.data,
                                        ctypes.byref(n))
    if rc:
        raise T2dError(rc, "psn_t2d_hungarian_match")
    return r[:n.value].tolist(), k[:n.value].tolist(), v[:n.value].tolist()


def result_with_tracker(trk: Tracker) -> dict:
    o = Object2D()
    rc = load().psn_t2d_result_with_tracker(ctypes.byref(trk), ctypes.byref(o))
    if rc:
        raise T2dError(rc, "psn_t2d_result_with_tracker")
    return object_dict(o)


def object_dict(o) -> dict:
    return {"id": o.id, "box": o.box.tuple(), "head": o.head.tuple(), "score": o.score,
            "prev": points(o.prev, o.num_prev), "curr": points(o.curr, o.num_curr)}


def matching_and_updating(dets: list[Detection], trackers: list[Tracker], cost, frame_idx: int, next_id: int,
                          match=None, cam_id: int = 0, cap=64):
    """psn_t2d_matching_and_updating -> (new active trackers, result dict, next id)."""
    L = load()
    da = (Detection * max(len(dets), 1))(*dets)
    ta = (Tracker * max(len(trackers), 1))(*trackers)
    c = np.ascontiguousarray(cost if cost is not None else np.zeros((0, 0)), np.float32)
    m = None if match is None else np.ascontiguousarray(match, np.int32)
    out = (Tracker * cap)()
    nout, nid = ctypes.c_int(), ctypes.c_uint(next_id)
    rb = ResultBuffers(cap, 1)
    rb.r.cam_id = cam_id
    rc = L.psn_t2d_matching_and_updating(da, len(dets), ta, len(trackers), c.ctypes.data if c.size else None,
                                         m.ctypes.data if m is not None else None, frame_idx, ctypes.byref(nid),
                                         out, cap, ctypes.byref(nout), ctypes.byref(rb.r))
    if rc:
        raise T2dError(rc, "psn_t2d_matching_and_updating")
    return list(out)[:nout.value], rb.to_dict(), nid.value


class Group:
    """psn_t2d_group: CPSNWhere_Tracker2D::Run of C cameras on one device,
    every camera's LK work batched into the same launches."""

    def __init__(self, width: int, height: int, cam_ids, device: int = 0, max_objects: int = 64):
        self._L = load()
        ids = (ctypes.c_uint * len(cam_ids))(*cam_ids)
        h = ctypes.c_void_p()
        rc = self._L.psn_t2d_group_create(device, len(cam_ids), ids, width, height, ctypes.byref(h))
        if rc:
            raise T2dError(rc, "psn_t2d_group_create")
        self._h = h
        self.ncams = len(cam_ids)
        self.width, self.height = width, height
        self.results = [ResultBuffers(max_objects, 1) for _ in range(self.ncams)]
        self._res = (Track2DResult * self.ncams)(*[r.r for r in self.results])
        self._keep = None

    def _check(self, rc, what):
        if rc:
            raise T2dError(rc, f"{what}: {self._L.psn_t2d_group_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.psn_t2d_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def lk_handle(self) -> int:
        return self._L.psn_t2d_group_lk_context(self._h)

    def push_frame(self, cam: int, img: np.ndarray):
        """Asynchronous upload of camera `cam`'s frame t (must stay alive until complete())."""
        assert img.flags["C_CONTIGUOUS"] and img.dtype == np.uint8
        ch = 1 if img.ndim == 2 else img.shape[2]
        self._check(self._L.psn_t2d_group_push_frame(self._h, cam, img.ctypes.data, img.shape[1] * ch, ch),
                    "push_frame")

    def push_frame_jpeg(self, cam: int, data):
        """Camera `cam`'s frame t as a baseline JPEG file (bytes or a uint8 array), decoded on the device."""
        self._check(self._L.psn_t2d_group_push_frame_jpeg(self._h, cam, data if isinstance(data, bytes) else
                                                          ctypes.c_void_p(data.ctypes.data), len(data)),
                    "push_frame_jpeg")

    def push_frame_device(self, cam: int, dev_ptr: int, stride: int, channels: int = 1):
        self._check(self._L.psn_t2d_group_push_frame_device(self._h, cam, ctypes.c_void_p(dev_ptr), stride, channels),
                    "push_frame_device")

    def records(self, dets_per_cam):
        """The ctypes records of one frame's detections (launch / complete_next accept them
        in place of the lists: a driver can build them outside its timed loop)."""
        if isinstance(dets_per_cam, tuple):
            return dets_per_cam
        arrs = [(Detection * max(len(d), 1))(*d) for d in dets_per_cam]
        ptrs = (ctypes.c_void_p * self.ncams)(*[ctypes.addressof(a) for a in arrs])
        nd = (ctypes.c_int * self.ncams)(*[len(d) for d in dets_per_cam])
        return arrs, ptrs, nd

    def launch(self, frame_idx: int, dets_per_cam, gridfast: bool = False, seed: int = 0):
        """dets_per_cam[c]: list of Detection records of camera c (kept alive until complete()).
        After complete_next(frame_idx, dets_per_cam, ...) the records given there are used
        (only the forward calls are enqueued here)."""
        ahead = getattr(self, "_ahead", None)
        if ahead is not None:
            arrs, ptrs, nd = ahead
        else:
            arrs, ptrs, nd = self.records(dets_per_cam)
        self._check(self._L.psn_t2d_group_launch(self._h, frame_idx, ptrs, nd, int(bool(gridfast)),
                                                 ctypes.c_uint32(seed & 0xffffffff)), "launch")
        self._ahead = None
        self._keep = (arrs, ptrs, nd)

    def complete_next(self, next_frame_idx: int, next_dets_per_cam, gridfast: bool = False, seed: int = 0,
                      raw: bool = False):
        """complete() of the current frame that launches frame next_frame_idx
        (psn_t2d_group_complete_next; that frame's images must be pushed already). The next
        call must be launch(next_frame_idx, next_dets_per_cam, gridfast, seed), which only
        confirms it."""
        arrs, ptrs, nd = self._keep
        nxt = self.records(next_dets_per_cam)
        rc = self._L.psn_t2d_group_complete_next(self._h, ptrs, nd, self._res, next_frame_idx, nxt[1], nxt[2],
                                                 int(bool(gridfast)), ctypes.c_uint32(seed & 0xffffffff))
        self._keep = None
        if rc:  # e.results: this frame's outputs when only the next frame's launch failed
            err = T2dError(rc, f"complete_next: {self._L.psn_t2d_group_last_error(self._h).decode()}")
            err.results = self._outputs(arrs, nd) if b"not launched" in self._L.psn_t2d_group_last_error(self._h) \
                else None
            raise err
        self._ahead = nxt
        return None if raw else self._outputs(arrs, nd)

    def _outputs(self, arrs, nd):
        out = []
        for c in range(self.ncams):
            self.results[c].r = self._res[c]
            out.append((list(arrs[c])[:nd[c]], self.results[c].to_dict()))
        return out

    def complete(self):
        """-> (per camera: list of output Detection records, result dict)."""
        arrs, ptrs, nd = self._keep
        self._check(self._L.psn_t2d_group_complete(self._h, ptrs, nd, self._res), "complete")
        self._keep = None
        out = []
        for c in range(self.ncams):
            self.results[c].r = self._res[c]
            out.append((list(arrs[c])[:nd[c]], self.results[c].to_dict()))
        return out

    def complete_raw(self):
        """complete() without converting the results (the caller packs self.result_struct(c))."""
        arrs, ptrs, nd = self._keep
        self._check(self._L.psn_t2d_group_complete(self._h, ptrs, nd, self._res), "complete")
        self._keep = None

    def result_struct(self, cam: int):
        return self._res[cam]

    def run(self, frame_idx: int, dets_per_cam, gridfast: bool = False, seed: int = 0):
        self.launch(frame_idx, dets_per_cam, gridfast, seed)
        return self.complete()

    def debug_host_times(self):
        """Mean host microseconds from the entry of complete to its phases since the last call
        (psn_t2d_group_debug_host_times)."""
        out = (ctypes.c_double * 6)()
        self._check(self._L.psn_t2d_group_debug_host_times(self._h, out), "debug_host_times")
        n = max(out[5], 1.0)
        keys = ["next_chains_enqueued", "device_done", "unpacked", "matched", "next_forward_enqueued"]
        m = (ctypes.c_double * 4)()
        self._check(self._L.psn_t2d_group_debug_host_match_times(self._h, m), "debug_host_match_times")
        parts = ["overlap_flags", "forward_costs", "assignment", "update_results"]
        return ({k: round(out[i] / n, 1) for i, k in enumerate(keys)} | {"completes": int(out[5])}
                | {"match_parts_us": {k: round(m[i] / n, 1) for i, k in enumerate(parts)}})

    def trackers(self, cam: int, cap: int = 256) -> list[Tracker]:
        out = (Tracker * cap)()
        n = ctypes.c_int()
        self._check(self._L.psn_t2d_group_trackers(self._h, cam, out, cap, ctypes.byref(n)), "trackers")
        return list(out)[:n.value]


# ---- stTrack2DResult formats (tracker2d_io.cpp) ----

class ResultBuffers:
    """A Track2DResult with caller-owned arrays (capacities for the readers)."""

    def __init__(self, cap_objects=64, cap_rects=64):
        self.objs = (Object2D * max(cap_objects, 1))()
        self.dets = (Rect * max(cap_rects, 1))()
        self.trks = (Rect * max(cap_rects, 1))()
        self.r = Track2DResult()
        self.r.objects = ctypes.cast(self.objs, ctypes.POINTER(Object2D))
        self.r.detection_rects = ctypes.cast(self.dets, ctypes.POINTER(Rect))
        self.r.tracker_rects = ctypes.cast(self.trks, ctypes.POINTER(Rect))
        self.r.cap_objects, self.r.cap_detection_rects, self.r.cap_tracker_rects = cap_objects, cap_rects, cap_rects

    @classmethod
    def from_dict(cls, d):
        b = cls(max(len(d["objects"]), 1), max(len(d["detection_rects"]), len(d["tracker_rects"]), 1))
        b.r.cam_id, b.r.frame_idx = d["cam_id"], d["frame_idx"]
        for i, o in enumerate(d["objects"]):
            ob = b.objs[i]
            ob.id = o["id"]
            ob.box, ob.head, ob.score = rect(*o["box"]), rect(*o["head"]), float(o["score"])
            for key, nk in (("prev", "num_prev"), ("curr", "num_curr")):
                pts = np.asarray(o[key], np.float32).reshape(-1, 2)
                setattr(ob, nk, len(pts))
                arr = getattr(ob, key)
                for k, (x, y) in enumerate(pts):
                    arr[k][0], arr[k][1] = x, y
        b.r.num_objects = len(d["objects"])
        for i, t in enumerate(d["detection_rects"]):
            b.dets[i] = rect(*t)
        for i, t in enumerate(d["tracker_rects"]):
            b.trks[i] = rect(*t)
        b.r.num_detection_rects, b.r.num_tracker_rects = len(d["detection_rects"]), len(d["tracker_rects"])
        return b

    def to_dict(self):
        r = self.r
        objs = [object_dict(r.objects[i]) for i in range(r.num_objects)]
        return {"cam_id": r.cam_id, "frame_idx": r.frame_idx, "objects": objs,
                "detection_rects": [r.detection_rects[i].tuple() for i in range(r.num_detection_rects)],
                "tracker_rects": [r.tracker_rects[i].tuple() for i in range(r.num_tracker_rects)]}


def write_result_txt(dirpath: str, result: dict):
    rc = load().psn_t2d_write_result_txt(dirpath.encode(), ctypes.byref(ResultBuffers.from_dict(result).r))
    if rc:
        raise T2dError(rc, "psn_t2d_write_result_txt")


def read_result_txt(dirpath: str, cam_id: int, frame_idx: int, cap_objects=64, cap_rects=64) -> dict:
    b = ResultBuffers(cap_objects, cap_rects)
    rc = load().psn_t2d_read_result_txt(dirpath.encode(), cam_id, frame_idx, ctypes.byref(b.r))
    if rc:
        raise T2dError(rc, "psn_t2d_read_result_txt")
    return b.to_dict()


def result_slot_bytes(max_objects: int, max_rects: int) -> int:
    return load().psn_t2d_result_slot_bytes(max_objects, max_rects)


def pack_result(result: dict, slot: np.ndarray):
    rc = load().psn_t2d_pack_result(ctypes.byref(ResultBuffers.from_dict(result).r), slot.ctypes.data, slot.nbytes)
    if rc:
        raise T2dError(rc, "psn_t2d_pack_result")


def unpack_result(slot: np.ndarray, cap_objects=64, cap_rects=64) -> dict:
    b = ResultBuffers(cap_objects, cap_rects)
    s = np.ascontiguousarray(slot, np.uint8)
    rc = load().psn_t2d_unpack_result(s.ctypes.data, s.nbytes, ctypes.byref(b.r))
    if rc:
        raise T2dError(rc, "psn_t2d_unpack_result")
    return b.to_dict()
