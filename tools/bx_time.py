#!/usr/bin/env python3
"""Isolated launch time of the box-window LK kernel (lk_kernel_bx) on the
Tracker2D shapes: 2048 points (the default bench's frame-set: 4 cameras x 512)
of 64x64 (backward chain steps) and of 64x160 (forward) windows, maxLevel 3,
the reference's criteria (30, 0.01), on the synthetic 1080p scene. Each launch
is timed with HIP events on the context stream (psn_lk_timing_launches); prints
the median / mean over `--reps` launches and a checksum of the outputs (the
same checksum across builds = the same results).

  python tools/bx_time.py --reps 40
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcmtt_opticalflow_amd import _lib, lk, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--shapes", default="64x64,64x160")
    ap.add_argument("--lib", default=None, help="a libpsn_lk.so build to time (default: the product library)")
    ap.add_argument("--variants", default="", help="context variants, e.g. lg_jr=0,large=1")
    args = ap.parse_args()
    variants = {k: int(v) for k, v in (kv.split("=") for kv in args.variants.split(",") if kv)}
    sc = synth.make_scene(0, 1920, 1080, args.points, nboxes=8)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(1)
    L = _lib.load(args.lib)
    out = {"points": args.points, "reps": args.reps, "variants": variants}
    with lk.LKContext(1920, 1080, ring_slots=2, max_level_cap=3, variants=variants) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        for shape in args.shapes.split(","):
            w, h = (int(v) for v in shape.split("x"))
            q = lk.make_query(1, 0, 0, args.points, lk.make_params((w, h), 3))
            for _ in range(3):
                res = ctx.track([q], pts)
            L.psn_lk_enable_timing(ctx.handle, args.reps + 1, 1)
            for _ in range(args.reps):
                res = ctx.track([q], pts)
            ms = np.array([m for m, _ in _lib.timing_launches(L, ctx.handle, args.reps + 1)])
            L.psn_lk_enable_timing(ctx.handle, 0, 1)
            dig = hashlib.sha1(b"".join(np.ascontiguousarray(a).tobytes() for a in res)).hexdigest()[:16]
            out[shape] = {"median_us": round(1e3 * float(np.median(ms)), 1), "mean_us": round(1e3 * float(ms.mean()), 1),
                          "min_us": round(1e3 * float(ms.min()), 1), "launches": int(ms.size), "out_sha": dig}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
