#!/usr/bin/env python3
"""Cost model of the LK kernel: device time vs. forced iteration count.

criteria = (COUNT, k, eps=0) with maxLevel 0 makes every point run exactly k
iterations (until it leaves the image), so the slope of kernel time over k is
the per-iteration critical path and the intercept the per-level fixed cost
(staging, Scharr, A-phase). `--texture strong|weak` selects whether the
exact-integer fast path or the ordered float chains carry the sums.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcmtt_opticalflow_amd import lk, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=512)
    ap.add_argument("--win", type=int, default=21)
    ap.add_argument("--win-h", type=int, default=0)
    ap.add_argument("--levels", type=int, default=1)
    ap.add_argument("--iters", default="0,1,2,4,8,16,30")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--textures", default="strong,weak")
    args = ap.parse_args()
    W, H = 1920, 1080
    out = []
    textures = args.textures.split(",")
    for texture in textures:
        sc = synth.make_scene(0, W, H, args.points)
        f0, f1 = sc.frame(0), sc.frame(1)
        if texture == "weak":  # 1/8 contrast: gradients 8x smaller, b-sums mostly exact
            f0 = (128 + (f0.astype(np.int32) - 128) // 8).astype(np.uint8)
            f1 = (128 + (f1.astype(np.int32) - 128) // 8).astype(np.uint8)
        pts = sc.points_at(0)
        with lk.LKContext(W, H, ring_slots=2, max_level_cap=max(args.levels - 1, 0)) as ctx:
            ctx.push_frame(0, f0)
            ctx.push_frame(1, f1)
            for k in [int(x) for x in args.iters.split(",")]:
                p = lk.make_params((args.win, args.win_h or args.win), args.levels - 1, criteria=(1, k, 0.0))
                q = lk.make_query(0, 1, 0, len(pts), p)
                ctx.track([q], pts)  # warm
                ctx.enable_timing(args.reps)
                for _ in range(args.reps):
                    ctx.track([q], pts)
                ts = ctx.timing_stats()
                us = 1e3 * ts["track_ms"] / ts["n_track"]
                out.append({"texture": texture, "iters": k, "us": round(us, 2)})
                print(json.dumps(out[-1]), flush=True)
    for texture in textures:
        xs = np.array([o["iters"] for o in out if o["texture"] == texture], float)
        ys = np.array([o["us"] for o in out if o["texture"] == texture], float)
        slope, icpt = np.polyfit(xs, ys, 1)
        print(json.dumps({"texture": texture, "us_per_iteration": round(slope, 3), "us_fixed": round(icpt, 2)}))


if __name__ == "__main__":
    main()
