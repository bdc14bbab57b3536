#!/usr/bin/env python3
"""Statistics of lk_kernel_bx's b-sum chains on the bench's Tracker2D workload
(analysis only): the oracle Tracker2D (oracle/tracker2d_oracle.py) runs one
camera of bench.py's default configuration, and every b-sum evaluation of its
LK calls goes through the binade-run model (oracle/chain_model.c):

  - how many evaluations take the exact fast path,
  - how long the serial walk of the binade-run fallback is (records + HARD
    terms of the longest chain), and how many records / HARD segments one
    wave of one chain needs (the kernel's LDS record capacity),
  - and that the model equals the sequential float sum on every chain.

  FRAMES=6 python tools/chain_stats.py
"""
import ctypes

CHAIN_LOG_ENTRIES = 25  # ORACLE_CHAIN_LOG_ENTRIES (oracle/lk_oracle.h)
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (analysis only)
import tracker2d_oracle as T2  # noqa: E402
from mcmtt_opticalflow_amd import synth  # noqa: E402

KEYS = ["evals", "fast_path", "mismatch", "walk_sum", "walk_max", "records", "hard_segs", "hard_terms",
        "max_wave_records", "max_wave_hard", "fallback_evals",
        "suffix_terms", "suffix_exact_steps", "suffix_exact_in_blocks16",
        "u14", "u15", "fb_evals", "walk_sum2", "walk_abort", "walk_mismatch", "serial_from_first", "hard_terms2",
        "serial_first_to_last", "threads_first_to_last", "threads_first_to_end"]


def main():
    frames = int(os.environ.get("FRAMES", "6"))
    upt = int(os.environ.get("UPT", "0"))
    W, H, npts, nboxes, period = 1920, 1080, 512, 8, 10
    sc = synth.make_scene(0, W, H, npts, nboxes=nboxes)
    L = oracle.lib()
    buf = (ctypes.c_longlong * CHAIN_LOG_ENTRIES)()
    L.oracle_set_chain_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.oracle_set_chain_log(ctypes.addressof(buf), upt)
    T2.NTHREADS = 1
    cam = T2.CameraTracker(0)
    for t in range(frames):
        f = t % (2 * (period - 1))
        f = f if f < period else 2 * (period - 1) - f
        gray = oracle.bgr2gray(synth.to_bgr(sc.frame(f)))
        bx = [T2.Rect(float(int(x)), float(int(y)), float(sc.box_w), float(sc.box_h)) for x, y in sc.box_at(f)]
        pts = sc.points_at(f)
        feats = [pts[sc.pt_box == k] for k in range(nboxes)]
        extra = [(T2.Rect(b.x + b.w / 4, b.y, b.w / 2, b.h / 8), ((b.x + b.w / 2) * 10.0, (b.y + b.h) * 10.0, 0.0),
                  1700.0) for b in bx]
        cam.run(gray, bx, feats, t, extra)
    L.oracle_set_chain_log(None, 0)
    s = dict(zip(KEYS, list(buf)[:len(KEYS)]))
    fb = max(s["fallback_evals"], 1)
    s["walk_mean"] = round(s["walk_sum"] / fb, 1)
    s["records_per_chain"] = round(s["records"] / (10 * fb), 2)
    s["hard_terms_per_eval"] = round(s["hard_terms"] / fb, 1)
    print(json.dumps(s, indent=1))
    _ = np


if __name__ == "__main__":
    main()
