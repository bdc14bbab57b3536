"""CPSNWhere_Tracker2D::Run of several cameras in one group (psn_t2d_group_*,
include/psn_tracker2d.h): every camera's backward chain steps and forward calls
share LK launches, frames are uploaded asynchronously into staging slots (frame
t+1 while frame t runs), and after the flow the matching, tracker update and
ResultWithTracker produce each camera's stTrack2DResult.

Checked against oracle/tracker2d_oracle.py's CameraTracker (the reference
schedule: one calcOpticalFlowPyrLK per detection per chain step and per tracker,
both pyramids rebuilt in each) bit for bit: detections (boxes, point sets),
result objects (ids, boxes, heads, featurePointsPrev/Curr) and the surviving
trackers. Parity with OpenCV itself is unpinned.
"""
import numpy as np
import pytest

from mcmtt_opticalflow_amd import synth
from mcmtt_opticalflow_amd import tracker2d as t2d

ORC = pytest.importorskip("tracker2d_oracle")

pytestmark = pytest.mark.gpu


def _bgr(gray, seed):
    """A BGR frame whose BGR2GRAY is computed by the oracle (exercises the fused ingest)."""
    rng = np.random.default_rng(seed)
    d = rng.integers(-6, 7, gray.shape + (3,))
    return np.clip(gray[..., None].astype(np.int32) + d, 0, 255).astype(np.uint8)


def _camera_dets(sc, t, rng, tiny=False):
    """Detections at frame t: integer boxes, head boxes, a 3D estimate, and
    stand-in GridFAST points inside the boxes; optionally a 2-px-wide detection
    with 3 points (dropped before its LK call, :744 -- its 2x2 window must not
    fail the frame)."""
    boxes, extra, feats = [], [], []
    for k, (bx, by) in enumerate(sc.box_at(t)):
        box = (float(np.floor(bx)), float(np.floor(by)), float(sc.box_w), float(sc.box_h))
        head = (box[0] + box[2] / 4, box[1], box[2] / 2, box[3] / 8)
        loc = (box[0] * 10.0, box[1] * 10.0, 0.0)
        n = int(rng.integers(20, 101))
        feats.append(np.stack([rng.uniform(box[0] + 2, box[0] + box[2] - 2, n),
                               rng.uniform(box[1] + 2, box[1] + box[3] - 2, n)], 1).astype(np.float32))
        boxes.append(box)
        extra.append((head, loc, 1700.0))
    if tiny:
        boxes.append((5.0, 5.0, 2.0, 30.0))
        extra.append(((5.0, 5.0, 2.0, 4.0), (0.0, 0.0, 0.0), 1700.0))
        feats.append(np.float32([[5.5, 9], [6, 12], [5.2, 20]]))
    return boxes, extra, feats


def _rois(boxes, W, H):
    out = []
    for b in boxes:
        x, y = max(0.0, b[0]), max(0.0, b[1])
        out.append((int(x), int(y), int(min(W - x - 1, b[2])), int(min(H - y - 1, b[3]))))
    return out


def _check_result(g_res, r_res, what):
    assert (g_res["cam_id"], g_res["frame_idx"]) == (r_res["cam_id"], r_res["frame_idx"]), what
    assert len(g_res["objects"]) == len(r_res["objects"]), what
    for go, ro in zip(g_res["objects"], r_res["objects"]):
        assert (go["id"], go["box"], go["head"], go["score"]) == (ro["id"], ro["box"], ro["head"], ro["score"]), what
        np.testing.assert_array_equal(go["prev"], ro["prev"], err_msg=what)
        np.testing.assert_array_equal(go["curr"], ro["curr"], err_msg=what)
    assert g_res["detection_rects"] == [] and g_res["tracker_rects"] == []


@pytest.mark.parametrize("ahead", [False, True, "two"])
@pytest.mark.parametrize("gridfast", [False, True])
@pytest.mark.parametrize("W,H,bw,bh", [(640, 480, 32, 80), (960, 540, 64, 160)])
def test_group_run_matches_oracle(oracle_mod, gridfast, W, H, bw, bh, ahead):
    """ahead: frame t+1's chains are launched by complete_next(t) before the host
    matches frame t (the pipelined driver of the bench); "two": besides, frames
    are staged two ahead (frame t+2 pushed while frame t runs, the bench's
    default driver)."""
    C, T = 3, 7
    scenes = [synth.make_scene(40 + c, W, H, 120, nboxes=3, box_w=bw, box_h=bh, max_speed=3.0) for c in range(C)]
    refs = [ORC.CameraTracker(cam_id=10 + c) for c in range(C)]
    rngs = [np.random.default_rng(500 + c) for c in range(C)]
    grays = [[sc.frame(t) for t in range(T)] for sc in scenes]
    bgrs = [[_bgr(grays[c][t], 100 * c + t) for t in range(T)] for c in range(C)]
    per_frame = [[_camera_dets(scenes[c], t, rngs[c], tiny=(c == 0)) for c in range(C)] for t in range(T)]
    g_frames = [[[t2d.make_detection(b, np.zeros((0, 2), np.float32) if gridfast else f, head=e[0],
                                     location=e[1], height=e[2]) for b, e, f in zip(*per_frame[t][c])]
                 for c in range(C)] for t in range(T)]
    n_obj = n_matched = 0
    stage = 2 if ahead == "two" else 1
    with t2d.Group(W, H, [10 + c for c in range(C)]) as g:
        for f in range(stage):
            for c in range(C):  # camera 1 ingests BGR, the others gray
                g.push_frame(c, bgrs[c][f] if c == 1 else grays[c][f])
        for t in range(T):
            per_cam = per_frame[t]
            g.launch(t, g_frames[t], gridfast=gridfast, seed=t)
            if t + stage < T:  # frame t+stage is uploaded while frame t runs
                for c in range(C):
                    g.push_frame(c, bgrs[c][t + stage] if c == 1 else grays[c][t + stage])
            if ahead and t + 1 < T:
                out = g.complete_next(t + 1, g_frames[t + 1], gridfast=gridfast, seed=t + 1)
            else:
                out = g.complete()
            for c in range(C):
                gray = oracle_mod.bgr2gray(bgrs[c][t]) if c == 1 else grays[c][t]
                boxes, extra, feats = per_cam[c]
                if gridfast:
                    feats, _ = oracle_mod.gridfast_detect(gray, _rois(boxes, W, H), seed=t)
                objs, _, r_res = refs[c].run(gray, [ORC.Rect(*b) for b in boxes], feats, t,
                                             [(ORC.Rect(*e[0]), e[1], e[2]) for e in extra])
                what = f"frame {t} camera {c}"
                g_out, g_res = out[c]
                for d, f in zip(g_out, feats):
                    np.testing.assert_array_equal(t2d.points(d.features, d.num_features), f, err_msg=what)
                valid = [d for d in g_out if d.valid]
                assert len(valid) == len(objs), what
                for d, o in zip(valid, objs):
                    assert [d.boxes[i].tuple() for i in range(d.num_boxes)] == [b.tuple() for b in o.boxes], what
                    assert d.num_sets == len(o.sets), what
                    for s in range(d.num_sets):
                        np.testing.assert_array_equal(t2d.points(d.sets[s], d.set_count[s]), o.sets[s], err_msg=what)
                _check_result(g_res, r_res, what)
                g_trk = g.trackers(c)
                assert [(x.id, x.duration, x.num_boxes) for x in g_trk] == \
                       [(x.id, x.duration, len(x.boxes)) for x in refs[c].active], what
                n_obj += len(g_res["objects"])
                n_matched += sum(1 for x in refs[c].active if x.duration > 1)
    assert n_obj > 20 and n_matched > 5  # the sequence creates and continues trackers


def test_group_ahead_protocol():
    """complete_next must be followed by the launch of the frame it announced."""
    W, H = 160, 120
    img = synth.texture(W, H, 3)
    d = [[t2d.make_detection((10, 10, 30, 60), np.float32([[20, 20], [25, 30], [30, 40], [22, 50]]))]]
    with t2d.Group(W, H, [0]) as g:
        g.push_frame(0, img)
        g.launch(0, d)
        g.push_frame(0, img)
        g.complete_next(1, d)
        with pytest.raises(t2d.T2dError):
            g.launch(2, d)  # not the announced frame
        g.launch(1, d)
        g.complete()
        g.push_frame(0, img)
        g.push_frame(0, img)  # two frames staged
        with pytest.raises(t2d.T2dError):
            g.push_frame(0, img)  # a third one has no slot
        g.run(2, d)
        g.run(3, d)
        with pytest.raises(t2d.T2dError):
            g.launch(4, d)  # nothing staged


def test_group_next_frame_failure_keeps_frame():
    """complete_next whose NEXT frame cannot launch (a 2-px-wide detection with 4
    features: CV_Assert(winSize > 2)) still delivers this frame's results; the
    next frame stays staged and a plain launch of it with valid detections gives
    the results of an undisturbed run."""
    W, H = 160, 120
    imgs = [synth.texture(W, H, 3 + t) for t in range(3)]
    good = [[[t2d.make_detection((10 + t, 10, 30, 60), np.float32([[20, 20], [25, 30], [30, 40], [22, 50]]))]]
            for t in range(3)]
    bad = [[t2d.make_detection((10, 10, 2, 30), np.float32([[11, 12], [11, 20], [11.5, 25], [11, 30]]))]]

    def plain():
        out = []
        with t2d.Group(W, H, [0]) as g:
            for t in range(3):
                g.push_frame(0, imgs[t])
                out.append(g.run(t, good[t])[0][1])
        return out

    ref = plain()
    with t2d.Group(W, H, [0]) as g:
        g.push_frame(0, imgs[0])
        g.launch(0, good[0])
        g.push_frame(0, imgs[1])
        with pytest.raises(t2d.T2dError) as e:
            g.complete_next(1, bad)
        assert e.value.results is not None
        r0 = e.value.results[0][1]
        g.launch(1, good[1])  # frame 1 is still staged
        r1 = g.complete()[0][1]
        g.push_frame(0, imgs[2])
        g.launch(2, good[2])
        r2 = g.complete()[0][1]
    for got, exp in zip([r0, r1, r2], ref):
        _check_result(got, exp, "after a failed next-frame launch")


def test_group_window_errors():
    """A detection whose box-width window the LK cannot run (2 px: CV_Assert(winSize > 2))
    fails the frame only when it has >= 4 features (:744)."""
    W, H = 160, 120
    img = synth.texture(W, H, 3)
    with t2d.Group(W, H, [0]) as g:
        g.push_frame(0, img)
        g.run(0, [[t2d.make_detection((10, 10, 30, 60), np.float32([[20, 20], [25, 30], [30, 40], [22, 50]]))]])
        g.push_frame(0, img)
        bad = t2d.make_detection((10, 10, 2, 30), np.float32([[11, 12], [11, 20], [11.5, 25], [11, 30]]))
        with pytest.raises(t2d.T2dError):
            g.run(1, [[bad]])
        g.push_frame(0, img)
        few = t2d.make_detection((10, 10, 2, 30), np.float32([[11, 12], [11, 20]]))
        (dets, res), = g.run(2, [[few]])
        assert dets[0].valid == 0 and res["objects"] == []


def test_group_unsupported_backward_window():
    """A detection box wider than 4095 px gives a backward window box.w x box.w of
    2^24+ px, past the LK's limits (psn_lk_window_supported): with >= 4 features
    the frame fails with PSN_LK_ERR_UNSUPPORTED at the host's window check, before
    any launch (the chain is flagged up front, not failed inside the LK pass), and
    the group runs the next frame normally."""
    W, H = 4400, 240
    img = synth.texture(W, H, 5)
    good = [[t2d.make_detection((40, 20, 60, 150), np.float32([[60, 40], [70, 80], [80, 120], [62, 100]]))]]
    with t2d.Group(W, H, [0]) as g:
        g.push_frame(0, img)
        g.run(0, good)
        g.push_frame(0, img)
        wide = t2d.make_detection((20, 20, 4200, 200), np.float32([[100, 40], [900, 80], [2000, 120], [4000, 100]]))
        with pytest.raises(t2d.T2dError) as e:
            g.run(1, [[wide]])
        assert e.value.code == -8  # PSN_LK_ERR_UNSUPPORTED
        g.push_frame(0, img)
        (dets, res), = g.run(2, good)
        assert len(dets) == 1


def test_group_failed_frame_after_regrow_matches_oracle(oracle_mod):
    """A frame that grows the chain buffers and then fails (a 2-px-wide detection
    with >= 4 features, CV_Assert(winSize > 2)) leaves the trackers of the frame
    before it; the next frame's forward calls then come from their host set 0
    (the device chain results were reallocated) -- bit for bit the reference,
    whose failed Run has pushed the frame and kept its trackers."""
    W, H, T = 640, 480, 4
    sc = synth.make_scene(77, W, H, 120, nboxes=3, box_w=32, box_h=80, max_speed=3.0)
    ref = ORC.CameraTracker(cam_id=5)
    rng = np.random.default_rng(9)
    grays = [sc.frame(t) for t in range(T)]
    per_frame = [_camera_dets(sc, t, rng) for t in range(T)]
    boxes, extra, feats = per_frame[1]
    for i in range(20):  # frame 1: enough detections to grow the chain buffers (16)
        x, y = float(rng.integers(10, W - 50)), float(rng.integers(10, H - 100))
        boxes.append((x, y, 32.0, 80.0))
        extra.append(((x + 8, y, 16.0, 10.0), (x, y, 0.0), 1700.0))
        feats.append(np.stack([rng.uniform(x + 2, x + 30, 30), rng.uniform(y + 2, y + 78, 30)], 1).astype(np.float32))
    boxes.append((300.0, 200.0, 2.0, 30.0))
    extra.append(((300.0, 200.0, 2.0, 4.0), (0.0, 0.0, 0.0), 1700.0))
    feats.append(np.float32([[300.5, 202], [301, 210], [300.2, 215], [300.7, 225]]))
    frames = [[t2d.make_detection(b, f, head=e[0], location=e[1], height=e[2])
               for b, e, f in zip(*per_frame[t])] for t in range(T)]
    with t2d.Group(W, H, [5]) as g:
        for t in range(T):
            g.push_frame(0, grays[t])
            boxes, extra, feats = per_frame[t]
            args = (grays[t], [ORC.Rect(*b) for b in boxes], feats, t, [(ORC.Rect(*e[0]), e[1], e[2]) for e in extra])
            if t == 1:
                with pytest.raises(t2d.T2dError):
                    g.run(t, [frames[t]])
                with pytest.raises(Exception):
                    ref.run(*args)
                continue
            (g_out, g_res), = g.run(t, [frames[t]])
            objs, _, r_res = ref.run(*args)
            _check_result(g_res, r_res, f"frame {t}")
            assert len([d for d in g_out if d.valid]) == len(objs), f"frame {t}"


@pytest.mark.parametrize("gridfast", [False, True])
def test_group_large_boxes_match_oracle(oracle_mod, gridfast):
    """PETS-scale boxes at 1280x720: forward windows 100x250 and 140x300 and the
    140x140 backward window run the large-window kernel, 100x100 the box
    kernel, in the same group launches -- bit for bit the reference schedule."""
    W, H, T = 1280, 720, 5
    sizes = [(100, 250), (140, 300)]
    C = len(sizes)
    scenes = [synth.make_scene(60 + c, W, H, 120, nboxes=2, box_w=bw, box_h=bh, max_speed=3.0)
              for c, (bw, bh) in enumerate(sizes)]
    refs = [ORC.CameraTracker(cam_id=c) for c in range(C)]
    rngs = [np.random.default_rng(700 + c) for c in range(C)]
    grays = [[sc.frame(t) for t in range(T)] for sc in scenes]
    per_frame = [[_camera_dets(scenes[c], t, rngs[c]) for c in range(C)] for t in range(T)]
    n_obj = 0
    with t2d.Group(W, H, list(range(C))) as g:
        for t in range(T):
            for c in range(C):
                g.push_frame(c, grays[c][t])
            frames = [[t2d.make_detection(b, np.zeros((0, 2), np.float32) if gridfast else f, head=e[0],
                                          location=e[1], height=e[2]) for b, e, f in zip(*per_frame[t][c])]
                      for c in range(C)]
            out = g.run(t, frames, gridfast=gridfast, seed=t)
            for c in range(C):
                boxes, extra, feats = per_frame[t][c]
                if gridfast:
                    feats, _ = oracle_mod.gridfast_detect(grays[c][t], _rois(boxes, W, H), seed=t)
                objs, _, r_res = refs[c].run(grays[c][t], [ORC.Rect(*b) for b in boxes], feats, t,
                                             [(ORC.Rect(*e[0]), e[1], e[2]) for e in extra])
                what = f"frame {t} camera {c}"
                g_out, g_res = out[c]
                valid = [d for d in g_out if d.valid]
                assert len(valid) == len(objs), what
                for d, o in zip(valid, objs):
                    assert [d.boxes[i].tuple() for i in range(d.num_boxes)] == [b.tuple() for b in o.boxes], what
                    for k in range(d.num_sets):
                        np.testing.assert_array_equal(t2d.points(d.sets[k], d.set_count[k]), o.sets[k], err_msg=what)
                _check_result(g_res, r_res, what)
                n_obj += len(g_res["objects"])
    assert n_obj >= 6


@pytest.mark.gpu
@pytest.mark.parametrize("coherent", [True, False])
@pytest.mark.parametrize("nbytes", [0, 5, 16, 1000, 4096 + 7, 300003])
def test_pass_copy_kernels(nbytes, coherent):
    """psn_t2d_upload_device / psn_t2d_download_device (the Tracker2D pass's
    input and result copies): byte-exact both ways through a pinned block, the
    16-B body and the byte tail, rejected when misaligned."""
    import ctypes

    import hiprt
    from mcmtt_opticalflow_amd import _lib

    L = _lib.load()
    vp = ctypes.c_void_p
    for f in (L.psn_t2d_upload_device, L.psn_t2d_download_device):
        f.argtypes = [vp, vp, ctypes.c_size_t, vp]
    H = hiprt.hip()
    H.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    H.hipHostFree.argtypes = [vp]
    flags = 0x40000000 if coherent else 0  # hipHostMallocCoherent / hipHostMallocDefault
    hin, hout = vp(), vp()
    assert H.hipHostMalloc(ctypes.byref(hin), max(nbytes, 16) + 16, flags) == 0
    assert H.hipHostMalloc(ctypes.byref(hout), max(nbytes, 16) + 16, flags) == 0
    try:
        rng = np.random.default_rng(nbytes)
        src = rng.integers(0, 256, nbytes, dtype=np.uint8)
        ctypes.memmove(hin.value, src.ctypes.data, nbytes)
        ctypes.memset(hout.value, 0xA5, max(nbytes, 16) + 16)
        dev = hiprt.DeviceBuffer(max(nbytes, 16) + 16)
        assert L.psn_t2d_upload_device(dev.addr, hin.value, nbytes, None) == 0
        assert L.psn_t2d_download_device(hout.value, dev.addr, nbytes, None) == 0
        assert H.hipDeviceSynchronize() == 0
        got = np.ctypeslib.as_array((ctypes.c_uint8 * (max(nbytes, 16) + 16)).from_address(hout.value)).copy()
        assert np.array_equal(got[:nbytes], src)
        assert np.all(got[nbytes:] == 0xA5)  # nothing written past the block
        if nbytes:
            assert L.psn_t2d_upload_device(dev.addr + 4, hin.value, nbytes, None) != 0
            assert L.psn_t2d_download_device(hout.value + 8, dev.addr, nbytes, None) != 0
        dev.free()
    finally:
        H.hipHostFree(hin)
        H.hipHostFree(hout)
