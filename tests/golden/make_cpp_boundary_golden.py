"""Fixtures of the compiled C++ boundary test (tests/test_cpp_boundary.py).

The inputs -- five 1280x720 BGR frames of one camera with four PETS-like
detections (synth.pets_box_sizes: forward windows up to 113x252 px, so the
box kernel and the large-window kernel both run) -- are regenerated from the
seeded synthetic scene by `inputs()`; the expected outputs are the reference's
FilePrintResult text files (PSNWhere_Tracker2D.cpp:1268-1334 format strings)
of oracle/tracker2d_oracle.py's CameraTracker replay of the same frames with
GridFAST features (oracle/gridfast_oracle.c, seed = frame index), written to
tests/golden/cpp_boundary/. Run in the build container:
    python tests/golden/make_cpp_boundary_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

W, H, T, CAM, NBOX = 1280, 720, 5, 7, 4
OUT = os.path.join(HERE, "cpp_boundary")


def inputs():
    """(bgr frames, per frame [(box, head)]) of the harness run."""
    from mcmtt_opticalflow_amd import synth

    sc = synth.make_scene(CAM, W, H, 4 * NBOX, nboxes=NBOX, box_dist="pets", max_speed=3.0)
    frames, dets = [], []
    for t in range(T):
        frames.append(synth.to_bgr(sc.frame(t)))
        per = []
        for k, (x, y) in enumerate(sc.box_at(t)):
            bw, bh = sc.box_size(k)
            box = (float(int(x)), float(int(y)), float(bw), float(bh))
            per.append((box, (box[0] + box[2] / 4, box[1], box[2] / 2, box[3] / 8)))
        dets.append(per)
    return frames, dets


def reference_text(r):
    """FilePrintResult's fprintf calls, in order (PSNWhere_Tracker2D.cpp:1279-1329)."""
    out = ["camIdx:%d\nframeIdx:%d\n" % (r["cam_id"], r["frame_idx"]), "numObjectInfos:%d{\n" % len(r["objects"])]
    for o in r["objects"]:
        out.append("\t{\n")
        out.append("\t\tid:%d\n" % o["id"])
        out.append("\t\tbox:(%f,%f,%f,%f)\n" % tuple(o["box"]))
        out.append("\t\thead:(%f,%f,%f,%f)\n" % tuple(o["head"]))
        out.append("\t\tscore:%f\n" % o["score"])
        for tag, pts in (("featurePointsPrev", o["prev"]), ("featurePointsCurr", o["curr"])):
            out.append("\t\t%s:%d,{" % (tag, len(pts)) + ",".join("(%f,%f)" % (float(x), float(y)) for x, y in pts)
                       + "}\n")
        out.append("\t}\n")
    out.append("}\n")
    out.append("detectionRects:0,{}\n")
    out.append("trackerRects:0,{}\n")
    return "".join(out)


def main():
    import oracle
    import tracker2d_oracle as T2

    frames, dets = inputs()
    ref = T2.CameraTracker(cam_id=CAM)
    os.makedirs(OUT, exist_ok=True)
    for t in range(T):
        gray = oracle.bgr2gray(frames[t])
        boxes = [b for b, _ in dets[t]]
        rois = []
        for b in boxes:  # rectROI = box.cropWithSize(cols, rows).cv() (:736)
            x, y = max(0.0, b[0]), max(0.0, b[1])
            rois.append((int(x), int(y), int(min(W - x - 1, b[2])), int(min(H - y - 1, b[3]))))
        feats, _ = oracle.gridfast_detect(gray, rois, seed=t)
        extra = [(T2.Rect(*h), ((b[0] + b[2] / 2) * 10.0, (b[1] + b[3]) * 10.0, 0.0), 1700.0) for b, h in dets[t]]
        _, _, res = ref.run(gray, [T2.Rect(*b) for b in boxes], feats, t, extra)
        name = "track2D_result_cam%d_frame%04d.txt" % (CAM, t)
        with open(os.path.join(OUT, name), "w") as f:
            f.write(reference_text(res))
        print(name, len(res["objects"]), "objects", sum(len(o["curr"]) for o in res["objects"]), "points")


if __name__ == "__main__":
    main()
