#!/usr/bin/env python3
"""Phase breakdown of the LK kernel from in-kernel s_memtime stamps.

Needs the diagnostic library (make -C mcmtt_opticalflow_amd/csrc stamps);
run as PSN_LK_LIB=.../libpsn_lk_stamps.so python tools/lk_stamps.py.
Stamps are shader-clock ticks; read the SHARES, not absolute time (stamping
perturbs the kernel).
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from mcmtt_opticalflow_amd import _lib, lk, synth  # noqa: E402
import hiprt  # noqa: E402

PH = ["slot_load", "stage", "scharr", "iwin", "a_reduce", "a_chain_eig", "iters"]


def main():
    npts = int(os.environ.get("NPTS", "512"))
    win = int(os.environ.get("WIN", "21"))
    sc = synth.make_scene(0, 1920, 1080, npts)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(0)
    L = _lib.load()
    st = hiprt.DeviceBuffer(npts * 64 * 8)
    with lk.LKContext(1920, 1080, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        rc = L.psn_lk_debug_set_stamps(ctx.handle, st.addr)
        assert rc == 0, "not a stamps build"
        q = lk.make_query(0, 1, 0, npts, lk.make_params((win, win), 3))
        for _ in range(3):
            ctx.track([q], pts)
        s = st.to_array((npts, 64), np.uint64).astype(np.int64)
    tot = s[:, 61] - s[:, 60]
    out = {"wg_cycles_mean": float(tot.mean()), "wg_cycles_max": float(tot.max()),
           "kernel_span_cycles": float(s[:, 61].max() - s[:, 60].min()),
           "start_spread_cycles": float(s[:, 60].max() - s[:, 60].min())}
    slow = int(np.argmax(tot))
    for lev in range(3, -1, -1):
        b = lev * 10
        d = np.diff(s[:, b:b + 8], axis=1)  # phases 0..6
        iters = s[:, b + 8]
        out[f"L{lev}"] = {
            "mean": {k: round(float(v), 1) for k, v in zip(PH, d.mean(0))},
            "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
            "cycles_per_iter": round(float(d[:, 6].sum() / max(iters.sum(), 1)), 1),
            "slowest_wg": {k: int(v) for k, v in zip(PH, d[slow])} | {"iters": int(iters[slow])},
        }
    it = s[:, 40:46]
    n_it = sum(s[:, lev * 10 + 8] for lev in range(4))
    tot_it = n_it.sum()
    out["iteration_phases_cycles_per_iter"] = {
        "products": round(float(it[:, 0].sum() / tot_it), 1), "reduce_barrier": round(float(it[:, 1].sum() / tot_it), 1),
        "chain_combine": round(float(it[:, 2].sum() / tot_it), 1), "solve": round(float(it[:, 3].sum() / tot_it), 1),
        "chain_path_fraction": round(float(it[:, 4].sum() / tot_it), 3), "restage_fraction": round(float(it[:, 5].sum() / tot_it), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
