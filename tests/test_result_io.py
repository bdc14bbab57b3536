"""stTrack2DResult formats: the reference's text
files written by CPSNWhere_Tracker2D::FilePrintResult
(psn_where/PSNWhere_Tracker2D.cpp:1268-1334) and read by
psn::Read2DTrackResultWithTxt (psn_where/PSNWhere_Utils.cpp:1148-1237), and the
exact binary slot that one rank per camera all-gathers into Associator3D.

The expected text is rendered here from the reference's fprintf format strings
(C "%f" = Python "%f": both correctly rounded to 6 decimals); the reader must
parse it as the reference does (fscanf "%f" into float). Host-only: no GPU.
"""
import os

import numpy as np
import pytest

from mcmtt_opticalflow_amd import tracker2d as t2d


def _result(rng, cam=2, frame=17, nobj=3, ndet=4, ntrk=2):
    objs = []
    for k in range(nobj):
        n1, n2 = int(rng.integers(0, 101)), int(rng.integers(0, 101))
        objs.append({"id": int(rng.integers(0, 1000)),
                     "box": tuple(float(v) for v in rng.uniform(0, 1900, 4)),
                     "head": tuple(float(v) for v in rng.uniform(0, 1900, 4)),
                     "score": float(rng.uniform(0, 1)),
                     "prev": rng.uniform(0, 1900, (n1, 2)).astype(np.float32),
                     "curr": rng.uniform(0, 1900, (n2, 2)).astype(np.float32)})
    return {"cam_id": cam, "frame_idx": frame, "objects": objs,
            "detection_rects": [tuple(float(v) for v in rng.uniform(0, 1000, 4)) for _ in range(ndet)],
            "tracker_rects": [tuple(float(v) for v in rng.uniform(0, 1000, 4)) for _ in range(ntrk)]}


def _reference_text(r):
    """FilePrintResult's fprintf calls, in order (PSNWhere_Tracker2D.cpp:1279-1329)."""
    out = ["camIdx:%d\nframeIdx:%d\n" % (r["cam_id"], r["frame_idx"]), "numObjectInfos:%d{\n" % len(r["objects"])]
    for o in r["objects"]:
        out.append("\t{\n")
        out.append("\t\tid:%d\n" % o["id"])
        out.append("\t\tbox:(%f,%f,%f,%f)\n" % o["box"])
        out.append("\t\thead:(%f,%f,%f,%f)\n" % o["head"])
        out.append("\t\tscore:%f\n" % o["score"])
        for tag, pts in (("featurePointsPrev", o["prev"]), ("featurePointsCurr", o["curr"])):
            out.append("\t\t%s:%d,{" % (tag, len(pts)) + ",".join("(%f,%f)" % (float(x), float(y)) for x, y in pts) + "}\n")
        out.append("\t}\n")
    out.append("}\n")
    for tag in ("detectionRects", "trackerRects"):
        rects = r["detection_rects"] if tag == "detectionRects" else r["tracker_rects"]
        out.append("%s:%d,{" % (tag, len(rects)) + ",".join("(%f,%f,%f,%f)" % t for t in rects) + "}\n")
    return "".join(out)


def test_writer_matches_reference_format(tmp_path):
    rng = np.random.default_rng(1)
    for nobj, ndet, ntrk in ((3, 4, 2), (0, 0, 0), (1, 1, 0)):
        r = _result(rng, nobj=nobj, ndet=ndet, ntrk=ntrk)
        t2d.write_result_txt(str(tmp_path) + os.sep, r)
        path = tmp_path / ("track2D_result_cam%d_frame%04d.txt" % (r["cam_id"], r["frame_idx"]))
        assert path.read_text() == _reference_text(r)


def test_reader_parses_reference_text(tmp_path):
    rng = np.random.default_rng(2)
    r = _result(rng, cam=5, frame=123)
    (tmp_path / "track2D_result_cam5_frame0123.txt").write_text(_reference_text(r))
    g = t2d.read_result_txt(str(tmp_path) + os.sep, 5, 123)
    f32 = lambda v: float(np.float32(float("%f" % v)))  # printed with %f, parsed into float
    assert len(g["objects"]) == len(r["objects"])
    for a, b in zip(g["objects"], r["objects"]):
        assert a["id"] == b["id"] and a["score"] == f32(b["score"])
        assert a["box"] == tuple(f32(v) for v in b["box"]) and a["head"] == tuple(f32(v) for v in b["head"])
        for key in ("prev", "curr"):
            exp = np.array([[f32(x), f32(y)] for x, y in b[key]], np.float32).reshape(-1, 2)
            np.testing.assert_array_equal(a[key], exp)
    assert g["detection_rects"] == [tuple(f32(v) for v in t) for t in r["detection_rects"]]
    assert g["tracker_rects"] == [tuple(f32(v) for v in t) for t in r["tracker_rects"]]


def test_reader_errors(tmp_path):
    with pytest.raises(t2d.T2dError):
        t2d.read_result_txt(str(tmp_path) + os.sep, 0, 0)  # missing file
    rng = np.random.default_rng(3)
    r = _result(rng, cam=0, frame=1, nobj=3)
    t2d.write_result_txt(str(tmp_path) + os.sep, r)
    with pytest.raises(t2d.T2dError):
        t2d.read_result_txt(str(tmp_path) + os.sep, 0, 1, cap_objects=2)  # capacity
    (tmp_path / "track2D_result_cam0_frame0002.txt").write_text("camIdx:0\nframeIdx:2\nnumObjectInfos:1{\n\tgarbage")
    with pytest.raises(t2d.T2dError):
        t2d.read_result_txt(str(tmp_path) + os.sep, 0, 2)


def test_slot_round_trip_is_exact():
    rng = np.random.default_rng(4)
    r = _result(rng, nobj=5, ndet=7, ntrk=3)
    nb = t2d.result_slot_bytes(8, 8)
    assert nb % 64 == 0
    slot = np.zeros(nb, np.uint8)
    t2d.pack_result(r, slot)
    g = t2d.unpack_result(slot)
    assert (g["cam_id"], g["frame_idx"]) == (r["cam_id"], r["frame_idx"])
    for a, b in zip(g["objects"], r["objects"]):
        assert (a["id"], a["box"], a["head"], a["score"]) == (b["id"], b["box"], b["head"], b["score"])
        np.testing.assert_array_equal(a["prev"], b["prev"])
        np.testing.assert_array_equal(a["curr"], b["curr"])
    assert g["detection_rects"] == r["detection_rects"] and g["tracker_rects"] == r["tracker_rects"]
    with pytest.raises(t2d.T2dError):
        t2d.pack_result(r, np.zeros(64, np.uint8))  # too small
    bad = slot.copy()
    bad[:4] = 0
    with pytest.raises(t2d.T2dError):
        t2d.unpack_result(bad)  # no magic
