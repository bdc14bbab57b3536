#!/usr/bin/env python3
"""Generate the committed golden fixtures tests/golden/*.npz.

There are NO reference fixtures for this path: the reference ships no tests
and its LK arithmetic lives in OpenCV 2.4.6, which is absent here (SURVEY.md
8c). These fixtures are therefore produced by this repo's CPU oracle
(oracle/lk_oracle.c) on deterministic synthetic inputs and pin it against
regressions; they do NOT pin it to OpenCV ("parity unpinned").

Each fixture holds the inputs (two u8 frames, points, call parameters) and
the expected calcOpticalFlowPyrLK outputs (nextPts, status, err) plus the
expected pyramid of the first frame.

    python tests/golden/make_golden.py      # rewrites the .npz files
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from mcmtt_opticalflow_amd import synth  # noqa: E402

CASES = {
    # (cam, W, H, npts, win, maxLevel, accum, flags, criteria, box)
    "kernel_21x21_3lvl": (11, 320, 240, 96, (21, 21), 2, oracle.ACCUM_SSE2, 0, (3, 30, 0.01), None),
    "tracker_box_32x80_scalar": (12, 256, 192, 48, (32, 80), 3, oracle.ACCUM_SCALAR, 0, (3, 30, 0.01), (32, 80)),
    "tracker_box_32x32_sse2": (13, 256, 192, 48, (32, 32), 3, oracle.ACCUM_SSE2, 0, (3, 30, 0.01), (32, 80)),
    "criteria_eps0_minEig": (14, 192, 160, 40, (9, 15), 3, oracle.ACCUM_SSE2, oracle.GET_MIN_EIGENVALS,
                             (1, 12, 0.0), None),
}


def make(name):
    cam, W, H, n, win, ml, accum, flags, crit, box = CASES[name]
    kw = dict(box_w=box[0], box_h=box[1]) if box else {}
    sc = synth.make_scene(cam, W, H, n, **kw)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(0)
    # border / outside points exercise the reflect-101 padding and status=0 paths
    pts = np.concatenate([pts, np.array([[0.5, 0.5], [W - 1.25, H - 0.5], [-3.0, 20.0], [W + 40.0, 8.0]],
                                        np.float32)])
    nxt, st, err = oracle.calc_optical_flow_pyr_lk(f0, f1, pts, win, ml, criteria=crit, flags=flags,
                                                   accum=accum, nthreads=1)
    eff = oracle.effective_max_level(W, H, win[0], win[1], ml)
    pyr = oracle.build_pyramid(f0, eff + 1)
    out = dict(prev_img=f0, next_img=f1, prev_pts=pts, win=np.array(win, np.int32),
               max_level=np.int32(ml), accum=np.int32(accum), flags=np.int32(flags),
               criteria=np.array(crit, np.float64), next_pts=nxt, status=st, err=err)
    for i, lv in enumerate(pyr):
        out[f"pyr{i}"] = lv
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    return name, int(st.sum()), len(st)


if __name__ == "__main__":
    for name in CASES:
        print(make(name))
