#!/usr/bin/env python3
"""Phase clocks of the box-window LK kernel (lk_kernel_bx) from the diagnostic
build (make -C mcmtt_opticalflow_amd/csrc stamps; run with
the stamps build, mcmtt_opticalflow_amd/lib/libpsn_lk_stamps.so). Tracker2D-like windows on the synthetic
1080p scene, the reference's default criteria (30, 0.01), maxLevel 3.
Prints per-workgroup mean / slowest cycles per phase (s_memtime ticks, thread
0's view) and the serial-chain fraction of the iterations.

  WIN=64 WINH=160 NPTS=630 python tools/bx_stamps.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))  # hiprt: the tests' HIP runtime helper

from mcmtt_opticalflow_amd import _lib, lk, synth  # noqa: E402
import hiprt  # noqa: E402

PHASES = ["level_setup", "a_window", "a_sums", "iter_head_solve", "b_main_pass", "b_publish_eval",
          "b_serial_products", "b_serial_chains", "b_results"]


def main():
    npts = int(os.environ.get("NPTS", "630"))
    w, h = int(os.environ.get("WIN", "64")), int(os.environ.get("WINH", "160"))
    sc = synth.make_scene(0, 1920, 1080, npts, nboxes=8)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(1)
    L = _lib.load(_lib.STAMPS_LIB_PATH)
    st = hiprt.DeviceBuffer(npts * 64 * 8)
    with lk.LKContext(1920, 1080, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        rc = L.psn_lk_debug_set_stamps(ctx.handle, st.addr)
        assert rc == 0, "not a stamps build"
        q = lk.make_query(1, 0, 0, npts, lk.make_params((w, h), 3))
        for _ in range(3):
            ctx.track([q], pts)
        s = st.to_array((npts, 64), np.uint64).astype(np.int64)
    tot = s[:, 15]
    slow = int(np.argmax(tot))
    ph = s[:, :9].copy()
    ph[:, 5] += s[:, 9]  # slot 9 splits b_publish_eval: publish (9) + barrier and eval (5)
    out = {"window": [w, h], "points": npts, "wg_cycles_mean": float(tot.mean()), "wg_cycles_max": int(tot.max()),
           "iterations_mean": float(s[:, 10].mean()), "iterations_max": int(s[:, 10].max()),
           "serial_b_fraction": round(float(s[:, 11].sum() / max(s[:, 10].sum(), 1)), 3),
           "mean": {k: round(float(v), 1) for k, v in zip(PHASES, ph.mean(0))},
           "slowest_wg": {k: int(v) for k, v in zip(PHASES, ph[slow])} | {"iters": int(s[slow, 10]),
                                                                            "serial": int(s[slow, 11])}}
    nt = max(s[:, 14].sum(), 1)
    out["serial_b_tiles_per_serial_iteration"] = round(float(s[:, 14].sum() / max(s[:, 11].sum(), 1)), 2)
    out["serial_b_per_tile_chain_lane_view"] = {"chain_sum": round(float(s[:, 12].sum() / nt), 1),
                                                "barrier_wait": round(float(s[:, 13].sum() / nt), 1)}
    it = max(s[:, 10].sum(), 1)
    out["per_iteration"] = {k: round(float(ph[:, i].sum() / it), 1) for i, k in enumerate(PHASES) if i >= 3}
    out["per_iteration"]["b_publish_only"] = round(float(s[:, 9].sum() / it), 1)  # inside b_publish_eval
    # residency (stamps 16-18: s_memrealtime at 100 MHz at the start / end, HW_ID and
    # XCC_ID): how many workgroups each CU held at once, and the idle CU time
    r0, r1, hw = s[:, 16], s[:, 17], s[:, 18]
    if r1.max() > 0:
        hwid, xcc = hw & 0xffffffff, hw >> 32
        cu = (xcc << 16) | (((hwid >> 13) & 7) << 8) | (((hwid >> 12) & 1) << 4) | ((hwid >> 8) & 15)
        t0 = int(r0.min())
        span = int(r1.max()) - t0
        conc, per_cu = [], []
        for c in np.unique(cu):
            m = cu == c
            ev = sorted([(int(a), 1) for a in r0[m]] + [(int(b), -1) for b in r1[m]])
            cur = mx = 0
            busy = last = 0
            for t, d in ev:
                if cur > 0:
                    busy += t - last
                cur += d
                last = t
                mx = max(mx, cur)
            dur = int((r1[m] - r0[m]).sum())
            per_cu.append((int(m.sum()), mx, dur / max(busy, 1), busy))
        arr = np.array(per_cu, float)
        out["residency"] = {"span_us": round(span / 100.0, 1), "cus": int(len(per_cu)),
                            "wgs_per_cu": [int(arr[:, 0].min()), float(arr[:, 0].mean()), int(arr[:, 0].max())],
                            "max_concurrent_per_cu": [int(arr[:, 1].min()), int(arr[:, 1].max())],
                            "mean_concurrency_while_busy": round(float(arr[:, 2].mean()), 3),
                            "cu_busy_frac_of_span": round(float(arr[:, 3].mean() / max(span, 1)), 3),
                            "wg_us_mean": round(float((r1 - r0).mean()) / 100.0, 1),
                            "wg_us_max": round(float((r1 - r0).max()) / 100.0, 1),
                            "clock_ghz": round(float(tot.mean() / max((r1 - r0).mean(), 1) / 10.0), 3),
                            "last_start_us": round((int(r0.max()) - t0) / 100.0, 1)}
        # per XCD: the static share of the grid (blockIdx round-robin) and when it ends
        xs = {}
        for x in np.unique(xcc):
            m = xcc == x
            xs[int(x)] = {"wgs": int(m.sum()), "end_us": round((int(r1[m].max()) - t0) / 100.0, 1),
                          "wg_us_sum_ms": round(float((r1[m] - r0[m]).sum()) / 1e5, 2)}
        out["residency"]["per_xcd"] = xs
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
