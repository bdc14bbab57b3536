#!/usr/bin/env python3
"""Host-side phase times of bench.py's default (pipelined) Tracker2D step
(diagnostic): Python-side time of launch (a confirmation after complete_next),
the frame pushes, complete_next and the result packing per frame-set, and the
C++ phases inside complete_next (psn_t2d_group_debug_host_times).
Usage: python tools/t2d_host_timing.py [steps]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from mcmtt_opticalflow_amd import tracker2d as t2d  # noqa: E402


def main():
    import torch

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    torch.cuda.set_device(0)
    args = bench.parse_args([])
    W, H, C, B = args.width, args.height, args.cameras, args.boxes
    pinned = bench.pinned_allocator()
    feeds = [bench.CameraFeed(c, args, pinned) for c in range(C)]
    group = t2d.Group(W, H, list(range(C)), device=0, max_objects=2 * B)
    slot_bytes = t2d.result_slot_bytes(2 * B, 1)
    send = pinned((C, slot_bytes))
    T = t2d.load()
    seq = [group.records([fd.detections(t2d, t) for fd in feeds]) for t in range(steps + 6)]
    for k, fd in enumerate(feeds):
        fd.push(group, k, 0)
    rows = []
    for t in range(steps + 5):
        if t == 5:
            group.debug_host_times()  # reset after the warm-up
        a = time.perf_counter()
        group.launch(t, seq[t])
        b = time.perf_counter()
        for k, fd in enumerate(feeds):
            fd.push(group, k, t + 1)
        c = time.perf_counter()
        group.complete_next(t + 1, seq[t + 1], raw=True)
        d = time.perf_counter()
        for k in range(C):
            T.psn_t2d_pack_result(ctypes.byref(group.result_struct(k)), send[k].ctypes.data, slot_bytes)
        e = time.perf_counter()
        if t >= 5:
            rows.append((b - a, c - b, d - c, e - d, e - a))
    r = np.array(rows) * 1e3
    names = ["launch (confirm)", "push x4", "complete_next", "pack", "total"]
    for i, n in enumerate(names):
        print(f"{n:32s} mean {r[:, i].mean():7.3f} ms  p50 {np.median(r[:, i]):7.3f}  max {r[:, i].max():7.3f}")
    print("complete_next phases (us from entry):", json.dumps(group.debug_host_times()))
    group.close()


if __name__ == "__main__":
    main()
