"""Tracker2D flow stage (libpsn_tracker2d.so, include/psn_tracker2d.h) against
the CPU restatement oracle/tracker2d_oracle.py.

CPU: every header symbol is exported; PSN_Rect arithmetic, BoxMatchingCost and
LocalSearchKLT agree with the restatement bit for bit on known answers and
seeded random cases (static points, clusters, ties, empty input).
GPU: a multi-frame sequence -- backward chains over the 4-frame ring, forward
tracking, matching costs, the majority gate -- through the C ABI (batched LK
launches on the device) equals the reference schedule run on the CPU oracle
(one calcOpticalFlowPyrLK per detection per step and per tracker), bit for bit.
Parity with OpenCV itself is unpinned.
"""
import ctypes
import math

import numpy as np
import pytest

from mcmtt_opticalflow_amd import synth
from mcmtt_opticalflow_amd import tracker2d as t2d

ORC = pytest.importorskip("tracker2d_oracle")


def test_symbols_exported():
    L = t2d.load()
    missing = [n for n in t2d.header_functions() if not hasattr(L, n)]
    assert not missing, missing


def _rand_rect(rng):
    return ORC.Rect(rng.uniform(-20, 300), rng.uniform(-20, 200), rng.integers(3, 90) + rng.uniform(0, 1) * (rng.random() < 0.3),
                    rng.integers(3, 200))


def test_rect_known_answers():
    L = t2d.load()
    a, b = t2d.rect(0, 0, 10, 10), t2d.rect(10, 0, 10, 10)
    assert L.psn_rect_overlap(a, b) == 0  # touching is not overlapping (strict <)
    assert L.psn_rect_overlap(a, t2d.rect(9.5, 9.5, 10, 10)) == 1
    cx, cy = ctypes.c_double(), ctypes.c_double()
    L.psn_rect_center(t2d.rect(1, 2, 5, 7), ctypes.byref(cx), ctypes.byref(cy))
    assert (cx.value, cy.value) == (1 + 3.0, 2 + 4.0)  # ceil(w/2)
    assert L.psn_rect_overlapped_area(a, b) == 0.0
    assert L.psn_rect_overlapped_area(a, t2d.rect(5, 5, 10, 10)) == 25.0
    assert L.psn_rect_contain(a, 0.0, 0.0) == 1 and L.psn_rect_contain(a, 10.0, 5.0) == 0
    assert L.psn_rect_distance(a, a) == 0.0
    assert L.psn_rect_distance(a, t2d.rect(3, 4, 10, 10)) == 0.5


def test_rect_ops_match_oracle():
    L = t2d.load()
    rng = np.random.default_rng(5)
    for _ in range(2000):
        p, q = _rand_rect(rng), _rand_rect(rng)
        cp, cq = t2d.rect(*p.tuple()), t2d.rect(*q.tuple())
        assert L.psn_rect_overlap(cp, cq) == int(p.overlap(q))
        assert L.psn_rect_distance(cp, cq) == p.distance(q)
        assert L.psn_rect_overlapped_area(cp, cq) == p.overlapped_area(q)
        assert L.psn_t2d_box_matching_cost(cp, cq) == ORC.box_matching_cost(p, q)
        px, py = np.float32(rng.uniform(-30, 320)), np.float32(rng.uniform(-30, 220))
        assert L.psn_rect_contain(cp, px, py) == int(p.contain(px, py))


def _klt_case(rng, n, kind):
    pre = rng.uniform(0, 100, (n, 2)).astype(np.float32)
    if kind == "static":
        d = rng.normal(0, 0.03, (n, 2))
    elif kind == "cluster":
        d = np.array([rng.uniform(-5, 5), rng.uniform(-5, 5)]) + rng.normal(0, 0.3, (n, 2))
        out = rng.random(n) < 0.3
        d[out] = rng.uniform(-20, 20, (out.sum(), 2))
    elif kind == "ties":
        d = rng.integers(-3, 4, (n, 2)).astype(np.float64)
    else:
        d = rng.uniform(-8, 8, (n, 2))
    cur = (pre + d).astype(np.float32)
    return pre, cur


@pytest.mark.parametrize("kind", ["static", "cluster", "ties", "uniform"])
def test_local_search_klt_matches_oracle(kind):
    rng = np.random.default_rng({"static": 1, "cluster": 2, "ties": 3, "uniform": 4}[kind])
    for trial in range(150):
        n = int(rng.integers(0, 101))
        pre, cur = _klt_case(rng, n, kind)
        box = (rng.uniform(0, 200), rng.uniform(0, 200), float(rng.integers(8, 80)), float(rng.integers(20, 200)))
        g_box, g_inl = t2d.local_search_klt(box, pre, cur)
        r_box, r_inl = ORC.local_search_klt(ORC.Rect(*box), pre, cur)
        assert g_box == r_box.tuple(), (kind, trial)
        assert g_inl == r_inl, (kind, trial)


def test_local_search_klt_window_edges():
    # neighbour counts at the window's edge (integer moves, integer windows
    # 0.2 * w), empty windows (w <= 0) and long runs of equal moves: the
    # two-pointer count of the host code must equal the restatement's double loop
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(1, 101))
        pre = rng.uniform(0, 100, (n, 2)).astype(np.float32)
        d = rng.integers(-4, 5, (n, 2)).astype(np.float64) * rng.choice([0.5, 1.0, 2.0])
        cur = (pre + d).astype(np.float32)
        w = float(rng.choice([0.0, -5.0, 5.0, 10.0, 15.0, 20.0, 25.0, 7.5, 12.5]))
        box = (rng.uniform(0, 200), rng.uniform(0, 200), w, 40.0)
        g_box, g_inl = t2d.local_search_klt(box, pre, cur)
        r_box, r_inl = ORC.local_search_klt(ORC.Rect(*box), pre, cur)
        assert g_box == r_box.tuple(), trial
        assert g_inl == r_inl, trial


def test_local_search_klt_semantics():
    # fewer than half the points move >= 0.1 px: the box stays and no inliers
    pre = np.zeros((10, 2), np.float32)
    cur = pre.copy()
    cur[:4] += 1.0
    box, inl = t2d.local_search_klt((10, 20, 30, 40), pre, cur)
    assert box == (10, 20, 30, 40) and inl == []
    # a common shift moves the box by the mode
    cur = pre + np.float32([2.0, -1.0])
    box, inl = t2d.local_search_klt((10, 20, 30, 40), pre, cur)
    assert box == (12.0, 19.0, 30, 40) and inl == list(range(10))
    box, inl = t2d.local_search_klt((1, 2, 3, 4), np.zeros((0, 2), np.float32), np.zeros((0, 2), np.float32))
    assert box == (1, 2, 3, 4) and inl == []


# ---------------------------------------------------------------------------
# GPU: multi-frame sequence through the C ABI vs the reference schedule
# ---------------------------------------------------------------------------

def _detections(sc, t, rng, W, H):
    """Integer detection boxes at frame t and GridFAST stand-in points inside
    them (seeded); one tiny detection with 3 points is dropped (:744)."""
    dets, feats = [], []
    for k, (bx, by) in enumerate(sc.box_at(t)):
        box = (float(np.floor(bx)), float(np.floor(by)), float(sc.box_w), float(sc.box_h))
        n = int(rng.integers(30, 101))
        pts = np.stack([rng.uniform(box[0] + 2, box[0] + box[2] - 2, n),
                        rng.uniform(box[1] + 2, box[1] + box[3] - 2, n)], 1).astype(np.float32)
        dets.append(box)
        feats.append(pts)
    dets.append((5.0, 5.0, 12.0, 30.0))
    feats.append(np.float32([[8, 9], [10, 12], [11, 20]]))
    return dets, feats


def _check_dets(g, r_objs, what):
    valid = [d for d in g if d.valid]
    assert len(valid) == len(r_objs), what
    for d, o in zip(valid, r_objs):
        assert d.overlap_other == int(o.overlap_other), what
        assert [d.boxes[i].tuple() for i in range(d.num_boxes)] == [b.tuple() for b in o.boxes], what
        assert d.num_sets == len(o.sets), what
        for s in range(d.num_sets):
            np.testing.assert_array_equal(t2d.points(d.sets[s], d.set_count[s]), o.sets[s], err_msg=what)


def _check_trackers(g, r_trk, g_cost, r_cost, what):
    for gt, rt in zip(g, r_trk):
        assert gt.updated == int(rt.updated), what
        assert [gt.boxes[i].tuple() for i in range(gt.num_boxes)] == [b.tuple() for b in rt.boxes], what
        np.testing.assert_array_equal(t2d.points(gt.features, gt.num_features), rt.features, err_msg=what)
        np.testing.assert_array_equal(t2d.points(gt.tracked, gt.num_tracked), rt.tracked, err_msg=what)
    np.testing.assert_array_equal(g_cost, r_cost, err_msg=what)


def _rect_roi(b, W, H):
    """rectROI = box.scale(1.0).cropWithSize(W, H).cv() (PSNWhere_Tracker2D.cpp:736)."""
    x, y = max(0.0, b[0]), max(0.0, b[1])
    return (int(x), int(y), int(min(W - x - 1, b[2])), int(min(H - y - 1, b[3])))


@pytest.mark.gpu
@pytest.mark.parametrize("merged,gridfast,device_chain,big,dev_frames",
                         [(False, False, False, False, False), (True, False, False, False, False),
                          (False, False, True, False, False), (True, False, True, False, False),
                          (True, True, True, False, False), (True, True, True, True, False),
                          (True, False, False, True, False), (True, True, True, True, True),
                          ("fused", True, True, False, False), ("fused", True, True, True, True),
                          ("fused", True, False, False, False)])
def test_tracker2d_sequence_matches_oracle(oracle_mod, merged, gridfast, device_chain, big, dev_frames):
    # merged == "fused": psn_t2d_track_frame_detect (GridFAST + chains + forward in one device pass)
    # big: 1080p-class boxes (64 x 160): 64 x 64 backward and 64 x 160 forward
    # windows run the tiled LK kernel (the counted launches included)
    W, H, T = (960, 540, 6) if big else (320, 240, 7)
    bw, bh = (64, 160) if big else (24, 60)
    sc = synth.make_scene(21, W, H, 120, nboxes=3, box_w=bw, box_h=bh, max_speed=3.0)
    rng = np.random.default_rng(77)
    ring = [None] * 4
    trackers = []  # oracle trackers (the harness's matching keeps both sides in sync)
    n_cost_finite = n_chain_steps = 0
    d_frames = []  # device copies of the frames (psn_t2d_push_frame_device), alive to the end
    with t2d.FlowTracker(W, H) as ft:
        ft.set_device_chain(device_chain)
        for t in range(T):
            img = sc.frame(t)
            if dev_frames:  # psn_t2d_push_frame_device from a frame already in HBM
                import hiprt  # tests/hiprt.py: the library's own HIP runtime
                d_frames.append(hiprt.DeviceBuffer.from_array(np.ascontiguousarray(img)))
                ft.push_frame_device(d_frames[-1].addr, W, 1)
            else:
                ft.push_frame(img)
            ring[-1] = img
            dets, feats = _detections(sc, t, rng, W, H)
            if gridfast:  # the detections' points from GridFAST on frame t (:734-757)
                feats, tots = oracle_mod.gridfast_detect(img, [_rect_roi(b, W, H) for b in dets], seed=t)
                if merged != "fused":
                    g_in = ft.detect_features([t2d.make_detection(b, np.zeros((0, 2), np.float32)) for b in dets],
                                              seed=t)
                    for d, f, n in zip(g_in, feats, tots):
                        np.testing.assert_array_equal(t2d.points(d.features, d.num_features), f, err_msg=f"frame {t}")
                        assert len(f) == min(int(n), 100)
            r_objs = ORC.backward_tracking(ring, [ORC.Rect(*b) for b in dets], feats)
            g_trk_in = [t2d.make_tracker([b.tuple() for b in tr.boxes], tr.features, tr.duration) for tr in trackers]
            r_cost = ORC.forward_tracking(ring, trackers, r_objs) if trackers else np.zeros((len(r_objs), 0), np.float32)
            g_det_in = [t2d.make_detection(b, f) for b, f in zip(dets, feats)]
            if merged == "fused":
                g_box_in = [t2d.make_detection(b, np.zeros((0, 2), np.float32)) for b in dets]
                g_dets, g_trk, g_cost = ft.track_frame_detect(g_box_in, g_trk_in, seed=t)
                for d, f in zip(g_dets, feats):
                    np.testing.assert_array_equal(t2d.points(d.features, d.num_features), f, err_msg=f"frame {t}")
            elif merged:
                g_dets, g_trk, g_cost = ft.track_frame(g_det_in, g_trk_in)
            else:
                g_dets = ft.backward(g_det_in)
                g_trk, g_cost = ft.forward(g_trk_in, g_dets) if g_trk_in else ([], np.zeros((len(r_objs), 0), np.float32))
            _check_dets(g_dets, r_objs, f"frame {t} backward")
            _check_trackers(g_trk, trackers, g_cost.reshape(r_cost.shape), r_cost, f"frame {t} forward")
            n_cost_finite += int(np.isfinite(r_cost).sum())
            n_chain_steps += sum(len(o.boxes) - 1 for o in r_objs)
            # harness matching (stands in for the Hungarian stage): tracker k <-> its cheapest finite detection
            new_trackers, used = [], set()
            for k, tr in enumerate(trackers):
                col = r_cost[:, k] if r_cost.size else np.zeros(0)
                cand = [d for d in np.argsort(col) if np.isfinite(col[d]) and d not in used]
                if not cand or tr.duration > 3:
                    continue
                d = int(cand[0])
                used.add(d)
                tr.duration += 1
                tr.boxes[-1] = r_objs[d].box
                tr.features = r_objs[d].sets[0].copy()
                tr.tracked = np.zeros((0, 2), np.float32)
                new_trackers.append(tr)
            for d, o in enumerate(r_objs):
                if d not in used:
                    new_trackers.append(ORC.Tracker([o.box], o.sets[0]))
            trackers = new_trackers
            ft.rotate()
            ring = ring[1:] + ring[:1]
    assert n_chain_steps > 10 and n_cost_finite > 3  # the sequence exercises chains and matches


@pytest.mark.gpu
def test_tracker2d_errors():
    with t2d.FlowTracker(160, 120) as ft:
        ft.push_frame(synth.texture(160, 120, 3))
        ft.rotate()
        ft.push_frame(synth.texture(160, 120, 3))
        d = t2d.make_detection((10, 10, 2, 30), np.float32([[12, 12], [13, 20], [11, 25], [12, 30]]))
        with pytest.raises(t2d.T2dError):  # window 2x2: CV_Assert(winSize > 2)
            ft.backward([d])
        bad = t2d.make_tracker([(10, 10, 20, 40)], np.zeros((5, 2), np.float32), duration=3)
        with pytest.raises(t2d.T2dError):
            ft.forward([bad], [])


# ---------------------------------------------------------------------------
# After the flow: assignment, tracker update, ResultWithTracker (:1038-1257)
# ---------------------------------------------------------------------------

def _rand_cost(rng, D, T):
    c = rng.uniform(0.0, 3.0, (D, T)).astype(np.float32)
    c[rng.random((D, T)) < 0.35] = np.inf
    return c


def _tie_cost(rng, D, T):
    """Few distinct values (many tied optima), non-finite entries, whole rows /
    columns without a finite entry."""
    c = rng.integers(0, 3, (D, T)).astype(np.float32) * np.float32(0.5)
    c[rng.random((D, T)) < 0.3] = np.inf
    if D and rng.random() < 0.3:
        c[int(rng.integers(0, D))] = np.inf
    if T and rng.random() < 0.3:
        c[:, int(rng.integers(0, T))] = -np.inf if rng.random() < 0.5 else np.inf
    return c


def test_hungarian_match_matches_oracle():
    """psn_t2d_hungarian_match (C++) == oracle/munkres_oracle.py (Python), both
    restating CPSNWhere_Hungarian::Match (helpers/PSNWhere_Hungarian.cpp:212-359):
    same pairs in the same order, including the reference's tie order, its
    FLT_MAX - sum infinity substitute, rows/columns without a finite entry
    (condensed out) and the NaN early-out (:78-81)."""
    import munkres_oracle as MO

    rng = np.random.default_rng(5)
    for trial in range(600):
        D, T = int(rng.integers(0, 9)), int(rng.integers(0, 9))
        c = _tie_cost(rng, D, T) if trial % 2 else _rand_cost(rng, D, T)
        g = t2d.hungarian_match(c)
        r = MO.hungarian_match(c)
        assert (g[0], g[1]) == (r[0], r[1]), (trial, c, g, r)
        assert np.array_equal(np.float32(g[2]), np.float32(r[2]))
    nan = np.float32([[1, 2], [np.nan, 0]])
    assert t2d.hungarian_match(nan) == ([], [], []) == MO.hungarian_match(nan)
    assert t2d.hungarian_match(np.full((3, 2), np.inf, np.float32)) == ([], [], [])


def test_hungarian_is_optimal_on_integer_costs():
    """On finite integer-valued costs every float operation is exact, so the
    Munkres restatements must reach the exhaustive minimum total cost."""
    import itertools

    import munkres_oracle as MO

    rng = np.random.default_rng(9)
    for trial in range(200):
        D, T = int(rng.integers(1, 6)), int(rng.integers(1, 6))
        c = rng.integers(0, 6, (D, T)).astype(np.float32)
        rows, cols, costs = t2d.hungarian_match(c)
        assert len(rows) == min(D, T) and len(set(rows)) == len(rows) and len(set(cols)) == len(cols)
        best = min(sum(float(c[d, p[d]]) for d in range(D)) for p in itertools.permutations(range(T), D)) \
            if D <= T else min(sum(float(c[p[t], t]) for t in range(T)) for p in itertools.permutations(range(D), T))
        assert sum(costs) == best, (trial, c)
        assert (rows, cols) == tuple(MO.hungarian_match(c)[:2])


def test_assign_matches_oracle():
    rng = np.random.default_rng(31)
    for trial in range(400):
        D, T = int(rng.integers(0, 6)), int(rng.integers(0, 6))
        c = _rand_cost(rng, D, T)
        assert t2d.assign(c) == ORC.assign(c), (trial, c)
    for trial in range(300):  # tie-heavy, up to the headline's 8 x 8 (and beyond)
        D, T = int(rng.integers(0, 13)), int(rng.integers(0, 13))
        c = _tie_cost(rng, D, T)
        assert t2d.assign(c) == ORC.assign(c), (trial, c)
    # all infinite: every pair sits at the substitute cost, nothing matches
    assert t2d.assign(np.full((3, 2), np.inf, np.float32)) == [-1, -1, -1]
    # the substitute (max + 100) can win over several finite pairs, as in the reference
    c = np.array([[90, np.inf, np.inf], [np.inf, 90, 0.0], [np.inf, 0.0, np.inf]], np.float32)
    assert t2d.assign(c) == ORC.assign(c)


def _rand_tracker(rng, id_, nb):
    boxes = [(float(rng.uniform(0, 300)), float(rng.uniform(0, 200)), 40.0, 100.0) for _ in range(nb)]
    heads = [(b[0] + 10, b[1], 20.0, 20.0) for b in boxes]
    f = rng.uniform(0, 300, (int(rng.integers(0, 30)), 2)).astype(np.float32)
    tr = t2d.make_tracker(boxes, f, duration=nb, heads=heads, id_=id_)
    tk = rng.uniform(0, 300, (int(rng.integers(0, len(f) + 1)), 2)).astype(np.float32)
    tr.num_tracked = len(tk)
    ctypes.memmove(tr.tracked, tk.ctypes.data, tk.nbytes)
    o = ORC.Tracker(boxes, f, duration=nb, heads=heads, id_=id_)
    o.tracked = tk
    return tr, o


def test_result_with_tracker_matches_oracle():
    rng = np.random.default_rng(8)
    for k in range(50):
        tr, o = _rand_tracker(rng, 100 + k, int(rng.integers(1, 6)))
        g, r = t2d.result_with_tracker(tr), ORC.result_with_tracker(o)
        assert (g["id"], g["box"], g["head"], g["score"]) == (r["id"], r["box"], r["head"], r["score"])
        np.testing.assert_array_equal(g["prev"], r["prev"])
        np.testing.assert_array_equal(g["curr"], r["curr"])


def test_matching_and_updating_matches_oracle():
    """Random post-forward states: matches pass or fail the 3D validation (distance
    600 mm, height 400 mm, duration 3); new trackers take ids in detection order;
    unmatched trackers end; result objects in the reference's order."""
    rng = np.random.default_rng(12)
    for trial in range(120):
        D, T = int(rng.integers(0, 6)), int(rng.integers(0, 6))
        g_trk, o_trk = zip(*[_rand_tracker(rng, 10 + i, int(rng.integers(1, 6))) for i in range(T)]) if T else ((), ())
        g_trk, o_trk = list(g_trk), list(o_trk)
        for gt, ot in zip(g_trk, o_trk):
            pos, h = tuple(rng.uniform(-500, 500, 3)), float(rng.uniform(1500, 2000))
            gt.last_position[:] = pos
            gt.height = h
            ot.last_position, ot.height = pos, h
            gt.time_start = ot.time_start = int(rng.integers(0, 5))
        g_det, o_det = [], []
        for i in range(D):
            box = (float(rng.uniform(0, 300)), float(rng.uniform(0, 200)), 40.0, 100.0)
            head = (box[0] + 12, box[1] + 1, 18.0, 22.0)
            loc, h = tuple(rng.uniform(-700, 700, 3)), float(rng.uniform(1400, 2300))
            f = rng.uniform(0, 300, (int(rng.integers(4, 40)), 2)).astype(np.float32)
            d = t2d.make_detection(box, np.zeros((0, 2), np.float32), head=head, location=loc, height=h)
            d.valid, d.num_boxes, d.num_sets, d.set_count[0] = 1, 1, 1, len(f)
            d.boxes[0] = t2d.rect(*box)
            ctypes.memmove(d.sets[0], f.ctypes.data, f.nbytes)
            g_det.append(d)
            od = ORC.DetectedObject(i, ORC.Rect(*box), ORC.Rect(*head), loc, h)
            od.sets = [f]
            o_det.append(od)
        cost = _rand_cost(rng, D, T)
        g_out, g_res, g_next = t2d.matching_and_updating(g_det, g_trk, cost, 7, 50, cam_id=3)
        o_act, o_objs, o_next = ORC.matching_and_updating(o_det, o_trk, ORC.assign(cost), 7, 50)
        assert g_next == o_next and len(g_out) == len(o_act) == len(g_res["objects"]) == len(o_objs), trial
        assert g_res["cam_id"] == 3 and g_res["frame_idx"] == 7
        for gt, ot in zip(g_out, o_act):
            assert (gt.id, gt.duration, gt.time_start, gt.time_end) == (ot.id, ot.duration, ot.time_start, ot.time_end)
            assert [gt.boxes[i].tuple() for i in range(gt.num_boxes)] == [b.tuple() for b in ot.boxes]
            assert [gt.heads[i].tuple() for i in range(gt.num_boxes)] == [b.tuple() for b in ot.heads]
            assert tuple(gt.last_position) == tuple(ot.last_position) and gt.height == ot.height
            np.testing.assert_array_equal(t2d.points(gt.features, gt.num_features), ot.features)
        for go, oo in zip(g_res["objects"], o_objs):
            assert (go["id"], go["box"], go["head"], go["score"]) == (oo["id"], oo["box"], oo["head"], oo["score"])
            np.testing.assert_array_equal(go["prev"], oo["prev"])
            np.testing.assert_array_equal(go["curr"], oo["curr"])


def test_matching_and_updating_rejects_repeated_tracker():
    """A caller-supplied match must be an assignment: two detections on one
    tracker would update and enqueue it twice (duplicate ids in the result)."""
    rng = np.random.default_rng(3)
    trk = [_rand_tracker(rng, 10 + i, 2)[0] for i in range(2)]
    dets = []
    for i in range(2):
        d = t2d.make_detection((10.0 * i, 5.0, 40.0, 100.0), np.zeros((0, 2), np.float32))
        f = np.float32([[1, 2], [3, 4], [5, 6], [7, 8]])
        d.valid, d.num_boxes, d.num_sets, d.set_count[0] = 1, 1, 1, len(f)
        ctypes.memmove(d.sets[0], f.ctypes.data, f.nbytes)
        dets.append(d)
    with pytest.raises(t2d.T2dError):
        t2d.matching_and_updating(dets, trk, None, 3, 0, match=[1, 1])
    t2d.matching_and_updating(dets, trk, None, 3, 0, match=[1, 0])
    t2d.matching_and_updating(dets, trk, None, 3, 0, match=[-1, -1])
