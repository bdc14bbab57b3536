"""oracle/tracker2d_oracle.py -- TEST INFRASTRUCTURE ONLY.

Plain-Python restatement of the Tracker2D flow stage of
psn_where/PSNWhere_Tracker2D.cpp, run in the reference's own schedule (one
calcOpticalFlowPyrLK per detection per chain step and per tracker, each on
full frames through oracle.calc_optical_flow_pyr_lk):
  local_search_klt        :452-554
  box_matching_cost       :600-613
  backward_tracking       :690-838
  forward_tracking        :851-1025
  assign / matching_and_updating / result_with_tracker   :1038-1164, :1231-1257
  CameraTracker.run       Run (:251-373) minus ingest and the height gate
and PSN_Rect arithmetic (PSNWhere_Types.h:112-182). Python floats are IEEE
doubles (the reference's double math); cv::Point2f differences are float32.
Only tests import this module.

PARITY UNPINNED (the reference ships no tests or fixtures for this path). The
assignment restates the reference's own Munkres, CPSNWhere_Hungarian
(oracle/munkres_oracle.py), so ties break in its order; that file is not
compiled here (it needs the MSVC CRT's _isnanf / _finitef).
"""
from __future__ import annotations

import math

import numpy as np

import munkres_oracle
import oracle as lk_oracle

MIN_FEATURES = 4     # PSN_2D_FEATURE_MIN_NUM_TRACK (:12)
MAX_FEATURES = 100   # PSN_2D_FEATURE_MAX_NUM_TRACK (:13)
INTERVAL = 4         # PSN_2D_BACKTRACKING_INTERVAL (:16)
SCALE = 1.0          # PSN_2D_OPTICALFLOW_SCALE (:18)
WIN_RATIO = 1.0      # PSN_2D_FEATURE_WIN_SIZE_RATIO (:15)


class Rect:
    __slots__ = ("x", "y", "w", "h")

    def __init__(self, x, y, w, h):
        self.x, self.y, self.w, self.h = float(x), float(y), float(w), float(h)

    def tuple(self):
        return (self.x, self.y, self.w, self.h)

    def center(self):  # ceil(w/2) (PSNWhere_Types.h:132)
        return (self.x + math.ceil(self.w / 2.0), self.y + math.ceil(self.h / 2.0))

    def scale(self, s):
        return Rect(self.x * s, self.y * s, self.w * s, self.h * s)

    def area(self):
        return self.w * self.h

    def contain(self, px, py):  # cv::Point2f overload
        px, py = float(np.float32(px)), float(np.float32(py))
        return px >= self.x and px < self.x + self.w and py >= self.y and py < self.y + self.h

    def overlap(self, a):  # strict '<' (:161-164)
        return (max(self.x + self.w, a.x + a.w) - min(self.x, a.x) < self.w + a.w) and \
               (max(self.y + self.h, a.y + a.h) - min(self.y, a.y) < self.h + a.h)

    def distance(self, a):  # (:165-170)
        dx = (self.x + self.w / 2.0) - (a.x + a.w / 2.0)
        dy = (self.y + self.h / 2.0) - (a.y + a.h / 2.0)
        dz = self.w - a.w
        return math.sqrt(dx * dx + dy * dy + dz * dz) / min(self.w, a.w)

    def overlapped_area(self, a):  # (:171-178)
        ow = min(self.x + self.w, a.x + a.w) - max(self.x, a.x)
        if 0.0 >= ow:
            return 0.0
        oh = min(self.y + self.h, a.y + a.h) - max(self.y, a.y)
        if 0.0 >= oh:
            return 0.0
        return ow * oh


def local_search_klt(pre_box: Rect, pre: np.ndarray, cur: np.ndarray):
    """:452-554 -> (box, inlier indices)."""
    pre = np.asarray(pre, np.float32).reshape(-1, 2)
    cur = np.asarray(cur, np.float32).reshape(-1, 2)
    n = len(pre)
    # vectors as doubles of the float32 differences (cv::Point2f - cv::Point2f),
    # each step elementwise IEEE double as the reference's scalar loops
    d = (cur - pre).astype(np.float64)
    keep = ~(np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) < 0.1 * SCALE)  # :481
    idx = np.nonzero(keep)[0]
    moving = d[idx]
    m = len(idx)
    if float(m) < float(n) * 0.5:
        return Rect(*pre_box.tuple()), []
    dxs, dys = np.sort(moving[:, 0]), np.sort(moving[:, 1])
    window = pre_box.w * 0.2 * SCALE
    # neighbour counts within the window (:505-537); the first maximum wins (strict <)
    nx = (np.abs(dxs[:, None] - dxs[None, :]) < window).sum(1)
    ny = (np.abs(dys[:, None] - dys[None, :]) < window).sum(1)
    ex = float(dxs[int(np.argmax(nx))]) if m and nx.max() > 0 else 0.0
    ey = float(dys[int(np.argmax(ny))]) if m and ny.max() > 0 else 0.0
    v = moving - np.array([ex, ey])
    inl = idx[np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) < window].tolist()  # :540-546
    box = Rect(*pre_box.tuple())
    box.x += ex
    box.y += ey
    return box, inl


def _norm(dx, dy):  # PSN_Point2D::norm_L2: sqrt(x*x + y*y)
    return math.sqrt(dx * dx + dy * dy)


def box_matching_cost(b1: Rect, b2: Rect) -> float:
    c1, c2 = b1.center(), b2.center()
    dx, dy = c1[0] - c2[0], c1[1] - c2[1]
    nom = math.sqrt(dx * dx + dy * dy)
    den = (b1.w + b2.w) / 2.0
    return (nom * nom) / (den * den)


# Schedule knobs (bench.py's cpu_baseline legs): OpenMP threads of every LK call
# (0: OMP_NUM_THREADS), and the shared-pyramid schedule -- each frame's
# pyramid built once and reused by every call, as the MI355X path does --
# instead of the reference's two pyramid builds per calcOpticalFlowPyrLK.
NTHREADS = 0
SHARED_PYRAMIDS = False
_pyramids = {}


def _pyramid(img):
    key = id(img)
    hit = _pyramids.get(key)
    if hit is None or hit[0] is not img:
        if len(_pyramids) > 64:
            _pyramids.clear()
        hit = (img, lk_oracle.build_pyramid_packed(img, 4))
        _pyramids[key] = hit
    return hit[1]


def _lk(prev_img, next_img, pts, win):
    pts = np.asarray(pts, np.float32).reshape(-1, 2)
    if len(pts) == 0:
        return np.zeros((0, 2), np.float32), np.zeros(0, np.uint8)
    if SHARED_PYRAMIDS:
        h, w = prev_img.shape
        nxt, st, _ = lk_oracle.lk_track_pyr(_pyramid(prev_img), _pyramid(next_img), w, h, pts, win, 3,
                                            nthreads=NTHREADS)
        return nxt, st
    nxt, st, _ = lk_oracle.calc_optical_flow_pyr_lk(prev_img, next_img, pts, win, 3,
                                                    nthreads=NTHREADS)  # err requested (:781)
    return nxt, st


class DetectedObject:
    def __init__(self, id_, box: Rect, head=None, location=(0.0, 0.0, 0.0), height=0.0):
        self.id = id_
        self.box = box
        self.head = head if head is not None else Rect(*box.tuple())
        self.location = tuple(float(v) for v in location)
        self.height = float(height)
        self.boxes = [box]
        self.sets = []
        self.overlap_other = False
        self.matched = False


def backward_tracking(ring, dets, features, extra=None):
    """:690-838. ring: 4 gray frames oldest first (None = empty slot), ring[-1]
    = frame t; dets: height-validated boxes; features: points at t per
    detection (after shuffle + cap); extra[i] = (head, location, height) of
    detection i (the caller's calibration). Returns m_vecDetection2D."""
    out = []
    for i, box in enumerate(dets):
        obj = DetectedObject(i, box, *(extra[i] if extra is not None else ()))
        f = np.asarray(features[i], np.float32).reshape(-1, 2)
        if len(f) < MIN_FEATURES:
            continue
        curr = f[:MAX_FEATURES].copy()
        cur_img = ring[-1]
        for s in range(1, INTERVAL):
            prev_img = ring[-1 - s]
            if prev_img is None:
                break
            rbox = box.scale(SCALE)
            win = int(rbox.w * WIN_RATIO)
            prev_pts, _status = _lk(cur_img, prev_img, curr, (win, win))  # status ignored (:787)
            new_rect, inl = local_search_klt(rbox, curr, prev_pts)
            if len(inl) < MIN_FEATURES:
                break
            obj.boxes.append(new_rect.scale(1.0 / SCALE))
            if not obj.sets:
                obj.sets.append(curr[inl].copy())
            curr = prev_pts[inl].copy()
            obj.sets.append(curr.copy())
            cur_img = prev_img
        if not obj.sets:
            obj.sets.append(curr.copy())
        out.append(obj)
    for a in range(len(out)):
        if out[a].overlap_other:
            continue
        for b in range(a + 1, len(out)):
            if out[a].box.overlap(out[b].box):
                out[a].overlap_other = True
                break
    return out


class Tracker:
    def __init__(self, boxes, features, duration=None, heads=None, id_=0):
        self.boxes = [Rect(*b) if not isinstance(b, Rect) else b for b in boxes]
        self.heads = [Rect(*b.tuple()) for b in self.boxes] if heads is None else \
            [Rect(*h) if not isinstance(h, Rect) else h for h in heads]
        self.duration = len(self.boxes) if duration is None else duration
        self.features = np.asarray(features, np.float32).reshape(-1, 2)
        self.tracked = np.zeros((0, 2), np.float32)
        self.updated = False
        self.id = id_
        self.time_start = self.time_end = self.time_last_update = 0
        self.last_position = (0.0, 0.0, 0.0)
        self.height = 0.0


def forward_tracking(ring, trackers, dets):
    """:851-1025. Returns the matching cost [len(dets) x len(trackers)] (float32)."""
    T, D = len(trackers), len(dets)
    cost = np.full((D, T), np.inf, np.float32)
    in_box = [[] for _ in range(D)]
    prev_img, cur_img = ring[-2], ring[-1]
    for t, tr in enumerate(trackers):
        rect = tr.boxes[-1].scale(SCALE)
        tr.tracked, status = _lk(prev_img, cur_img, tr.features, (int(rect.w * WIN_RATIO), int(rect.h * WIN_RATIO)))
        keep = [i for i in range(len(status)) if status[i]]
        v_prev, v_curr = tr.features[keep].copy(), tr.tracked[keep].copy()
        tr.updated = False
        if len(v_curr) < MIN_FEATURES:
            continue
        new_box, _ = local_search_klt(tr.boxes[-1].scale(SCALE), v_prev, v_curr)
        new_box = new_box.scale(1.0 / SCALE)
        tr.boxes.append(new_box)
        tr.heads.append(tr.heads[-1])  # :896
        tr.updated = True
        for d, det in enumerate(dets):
            if not new_box.overlap(det.box):
                continue
            for p in tr.tracked:  # the raw LK output (:914-918)
                if det.box.contain(p[0], p[1]):
                    in_box[d].append(t)
            box_cost = 0.0
            length = min(INTERVAL, min(len(tr.boxes), len(det.boxes)))
            tb = tr.duration
            for b in range(length):
                if not 0 <= tb < len(tr.boxes):  # past a failed frame: undefined in the reference (:948-952)
                    box_cost = math.inf
                    break
                db, tbx = det.boxes[b], tr.boxes[tb]
                if (not db.overlap(tbx) or 1.0 < db.distance(tbx)
                        or 0.3 > db.overlapped_area(tbx) / min(db.area(), tbx.area())
                        or 0.5 * max(db.w, tbx.w) < _norm(db.center()[0] - tbx.center()[0],
                                                           db.center()[1] - tbx.center()[1])):
                    box_cost = math.inf
                    break
                box_cost += box_matching_cost(tbx, db)
                tb -= 1
            if box_cost == math.inf:
                continue
            box_cost /= float(length)
            cost[d, t] = np.float32(box_cost)
        tr.features, tr.tracked = v_prev, v_curr
    for d in range(D):
        f = in_box[d]
        if not f:
            continue
        n_major = n_cur = 0
        cur = f[0]
        for k in range(len(f)):
            if cur == f[k]:
                n_cur += 1
                continue
            if n_cur > n_major:
                n_major = n_cur
            cur = f[k]
            n_cur = 0
        if f[0] == cur:
            n_major = n_cur
        if float(n_major) > float(len(f)) * 0.5:
            continue
        cost[d, :] = np.inf
    return cost


# ---------------------------------------------------------------------------
# After the flow: Track2D_MatchingAndUpdating (:1038-1164), ResultWithTracker
# ---------------------------------------------------------------------------

def assign(cost: np.ndarray) -> list:
    """:1040-1064 with the reference's Munkres (oracle/munkres_oracle.py): the
    tracker index per detection or -1."""
    return munkres_oracle.assign(cost)


def result_with_tracker(tr: Tracker) -> dict:
    """:1231-1257 (PSN_2D_DEBUG_DISPLAY_SCALE 1.0)."""
    return {"id": tr.id, "box": tr.boxes[-1].tuple(), "head": tr.heads[-1].tuple(), "score": 0.0,
            "prev": np.asarray(tr.features, np.float32).reshape(-1, 2).copy(),
            "curr": np.asarray(tr.tracked, np.float32).reshape(-1, 2).copy()}


def matching_and_updating(dets, active, match, frame_idx, next_id):
    """:1062-1164 -> (new active queue, result objects, next id)."""
    objects, nxt = [], []
    for d, det in enumerate(dets):
        t = match[d]
        if t < 0:
            continue
        tr = active[t]
        dist = math.sqrt(sum((det.location[k] - tr.last_position[k]) ** 2 for k in range(3)))
        if dist > 600.0 or abs(det.height - tr.height) > 400.0 or tr.duration > 3:
            continue
        det.matched = True
        tr.time_end = tr.time_last_update = frame_idx
        tr.duration = tr.time_end - tr.time_start + 1
        tr.boxes[-1] = det.box
        tr.heads[-1] = det.head
        tr.last_position, tr.height = det.location, det.height
        nxt.append(tr)
        objects.append(result_with_tracker(tr))
        tr.features = det.sets[0].copy()
        tr.tracked = np.zeros((0, 2), np.float32)
    for det in dets:
        if det.matched:
            continue
        tr = Tracker([det.box], det.sets[0], duration=1, heads=[det.head], id_=next_id)
        next_id += 1
        tr.time_start = tr.time_end = tr.time_last_update = frame_idx
        tr.last_position, tr.height = det.location, det.height
        nxt.append(tr)
        objects.append(result_with_tracker(tr))
    return nxt, objects, next_id


class CameraTracker:
    """One camera's CPSNWhere_Tracker2D::Run state (ring, active trackers,
    tracker ids) in the reference schedule."""

    def __init__(self, cam_id=0):
        self.cam_id = cam_id
        self.ring = [None] * INTERVAL
        self.active = []
        self.next_id = 0

    def run(self, frame, dets, features, frame_idx, extra=None):
        """-> (m_vecDetection2D, matching cost [D x T], result dict)."""
        self.ring = self.ring[1:] + [frame]
        objs = backward_tracking(self.ring, dets, features, extra)
        trackers = list(self.active)
        cost = forward_tracking(self.ring, trackers, objs) if trackers else np.zeros((len(objs), 0), np.float32)
        match = assign(cost)
        self.active, objects, self.next_id = matching_and_updating(objs, trackers, match, frame_idx, self.next_id)
        return objs, cost, {"cam_id": self.cam_id, "frame_idx": frame_idx, "objects": objects,
                            "detection_rects": [], "tracker_rects": []}
