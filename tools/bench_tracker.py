#!/usr/bin/env python3
"""Tracker2D-mode timing: the per-frame flow stage of CPSNWhere_Tracker2D::Run
as the reference drives it (box-derived windows, not the 21x21 kernel runs
of bench.py), on synthetic video:

  push frame t (ingest + pyramid)                       :256-263
  GridFAST features of every detection + shuffle/cap     :734-757
  backward chains (3 LK steps + LocalSearchKLT each)     :763-811
  forward LK of every tracker + matching score           :851-1025

Detections are the scene's boxes at frame t; the trackers of frame t are the
detections of frame t-1 (a stand-in for the Hungarian step, which is not on
the flow path). Reports Tracker2D frames/s per camera with the LocalSearchKLT
steps on the device (one host sync per frame) and on the host (a sync per
chain step).

  python tools/bench_tracker.py [--width 1920 --height 1080 --boxes 8 --frames 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcmtt_opticalflow_amd import synth  # noqa: E402
from mcmtt_opticalflow_amd import tracker2d as t2d  # noqa: E402


def run(args, device_chain: bool):
    W, H = args.width, args.height
    sc = synth.make_scene(0, W, H, 64 * args.boxes, nboxes=args.boxes)
    period = 10
    frames = [sc.frame(t) for t in range(period)]

    def ping(t):
        m = t % (2 * (period - 1))
        return m if m < period else 2 * (period - 1) - m

    stats = {"chains": 0, "features": 0, "tracked": 0}
    stage = {"push_ms": 0.0, "gridfast_ms": 0.0, "track_frame_ms": 0.0}
    with t2d.FlowTracker(W, H) as ft:
        ft.set_device_chain(device_chain)
        prev_objs = []
        t0 = None
        for t in range(args.warmup + args.frames):
            if t == args.warmup:
                t0 = time.perf_counter()
            ta = time.perf_counter()
            ft.push_frame(frames[ping(t)])
            tb = time.perf_counter()
            boxes = [(float(np.floor(x)), float(np.floor(y)), float(sc.box_w), float(sc.box_h))
                     for x, y in sc.box_at(ping(t))]
            dets = ft.detect_features([t2d.make_detection(b, np.zeros((0, 2), np.float32)) for b in boxes], seed=t)
            trackers = [t2d.make_tracker([b], f) for b, f in prev_objs]
            tc = time.perf_counter()
            dets_out, trk_out, _ = ft.track_frame(dets, trackers)
            td = time.perf_counter()
            if t >= args.warmup:
                stage["push_ms"] += 1e3 * (tb - ta)
                stage["gridfast_ms"] += 1e3 * (tc - tb)
                stage["track_frame_ms"] += 1e3 * (td - tc)
            prev_objs = [(d.box.tuple(), t2d.points(d.sets[0], d.set_count[0])) for d in dets_out
                         if d.valid and d.set_count[0] >= 4]
            if t >= args.warmup:
                stats["chains"] += sum(d.num_boxes - 1 for d in dets_out if d.valid)
                stats["features"] += sum(d.num_features for d in dets)
                stats["tracked"] += sum(tr.num_tracked for tr in trk_out)
            ft.rotate()
        dt = time.perf_counter() - t0
    return {"fps": args.frames / dt, "ms_per_frame": 1e3 * dt / args.frames,
            **{k: v / args.frames for k, v in stats.items()}, **{k: v / args.frames for k, v in stage.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--boxes", type=int, default=8)
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=8)
    args = ap.parse_args()
    out = {"workload": f"Tracker2D flow stage, {args.width}x{args.height}, {args.boxes} detections/frame, "
                       "GridFAST features, backward chains + forward LK, box-derived windows",
           "device_chain": run(args, True), "host_chain": run(args, False)}
    out["device_vs_host"] = round(out["device_chain"]["fps"] / out["host_chain"]["fps"], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
