#!/usr/bin/env python3
"""Phase clocks of the large-window LK kernel (lk_kernel_lg) from the diagnostic
build (make -C mcmtt_opticalflow_amd/csrc stamps): one window shape on the
synthetic 1080p scene (the kernel forced with variant large=1), per-point mean /
slowest s_memtime ticks per phase, iterations, fallback fraction; and the
isolated launch time of the product build for the same queries.

  WIN=100 WINH=250 NPTS=512 python tools/lg_stamps.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mcmtt_opticalflow_amd import _lib, lk, synth  # noqa: E402
import hiprt  # noqa: E402

PHASES = ["a_values", "a_runs_check_chains", "main_pass", "publish_check_eval", "fb_setup", "fb_tiles", "results"]


def main():
    npts = int(os.environ.get("NPTS", "512"))
    w, h = int(os.environ.get("WIN", "100")), int(os.environ.get("WINH", "250"))
    variants = {"large": 1}
    if os.environ.get("LG_LDS"):
        variants["lg_lds"] = int(os.environ["LG_LDS"])
    if os.environ.get("LG_JR"):
        variants["lg_jr"] = int(os.environ["LG_JR"])
    fw, fh = (3840, 2160) if os.environ.get("UHD") else (1920, 1080)
    levels = int(os.environ.get("LEVELS", "4" if fw > 1920 else "3"))
    sc = synth.make_scene(0, fw, fh, npts, nboxes=8, box_w=w, box_h=h)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(1)
    L = _lib.load(_lib.STAMPS_LIB_PATH)
    st = hiprt.DeviceBuffer(npts * 64 * 8)
    with lk.LKContext(fw, fh, ring_slots=2, max_level_cap=levels, variants=variants) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        rc = L.psn_lk_debug_set_stamps(ctx.handle, st.addr)
        assert rc == 0, "not a stamps build"
        q = lk.make_query(1, 0, 0, npts, lk.make_params((w, h), levels))
        for _ in range(2):
            ctx.track([q], pts)
        s = st.to_array((npts, 64), np.uint64).astype(np.int64)
        L.psn_lk_enable_timing(ctx.handle, 11, 1)
        for _ in range(10):
            ctx.track([q], pts)
        ms = [m for m, _ in _lib.timing_launches(L, ctx.handle, 11)]
    tot = s[:, 15]
    it = max(int(s[:, 10].sum()), 1)
    out = {"window": [w, h], "points": npts, "variants": variants,
           "launch_us_median_stamps_build": round(1e3 * float(np.median(ms)), 1),
           "wg_cycles_mean": float(tot.mean()), "wg_cycles_max": int(tot.max()),
           "iterations_mean": float(s[:, 10].mean()), "fallback_fraction": round(float(s[:, 11].sum() / it), 3),
           "mean": {k: round(float(v), 1) for k, v in zip(PHASES, s[:, :7].mean(0))},
           "a_values_split": {k: round(float(s[:, i].mean()), 1) for i, k in [(7, "stage"), (9, "quads")]},
           "fb_tiles_split": {k: round(float(s[:, i].sum() / max(int(s[:, 11].sum()), 1)), 1) for i, k in [(16, "pre"), (17, "chain_sums"), (18, "pad"), (13, "barrier"), (14, "tiles")]},
           "per_iteration": {k: round(float(s[:, i].sum() / it), 1) for i, k in enumerate(PHASES) if i >= 2},
           # every slot: mean ticks per point (slots 10, 11, 14 are counts)
           "slots_mean": [round(float(v), 1) for v in s[:, :24].mean(0)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
