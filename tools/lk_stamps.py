#!/usr/bin/env python3
"""Phase breakdown of the LK kernel from in-kernel s_memtime stamps.

Needs the diagnostic library (make -C mcmtt_opticalflow_amd/csrc stamps);
run as the stamps build, mcmtt_opticalflow_amd/lib/libpsn_lk_stamps.so python tools/lk_stamps.py.
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
sys.path.insert(0, os.path.join(ROOT, "tests"))  # hiprt: the tests' HIP runtime helper

from mcmtt_opticalflow_amd import _lib, lk, synth  # noqa: E402
import hiprt  # noqa: E402

PRO = ["prologue_dma", "scharr_all", "a_products_reduce", "a_chains_eig"]  # stamps 60->50->51->52->53
PH = ["level_setup_j_stage", "window_load", "iters"]  # per level: 0->1->2->7


def main():
    npts = int(os.environ.get("NPTS", "512"))
    win = int(os.environ.get("WIN", "21"))
    sc = synth.make_scene(0, 1920, 1080, npts)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(0)
    L = _lib.load(_lib.STAMPS_LIB_PATH)
    st = hiprt.DeviceBuffer(npts * 64 * 8)
    with lk.LKContext(1920, 1080, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        rc = L.psn_lk_debug_set_stamps(ctx.handle, st.addr)
        assert rc == 0, "not a stamps build"
        ovl = int(os.environ.get("ST_OVL", "1"))
        L.psn_lk_debug_set_variant(ctx.handle, _lib.VARIANTS["st_ovl"], ovl)
        q = lk.make_query(0, 1, 0, npts, lk.make_params((win, win), 3))
        for _ in range(3):
            ctx.track([q], pts)
        s = st.to_array((npts, 64), np.uint64).astype(np.int64)
    tot = s[:, 61] - s[:, 60]
    out = {"wg_cycles_mean": float(tot.mean()), "wg_cycles_max": float(tot.max()),
           "kernel_span_cycles": float(s[:, 61].max() - s[:, 60].min()),
           "start_spread_cycles": float(s[:, 60].max() - s[:, 60].min())}
    slow = int(np.argmax(tot))
    pro = np.stack([s[:, 50] - s[:, 60], s[:, 51] - s[:, 50], s[:, 52] - s[:, 51], s[:, 53] - s[:, 52]], 1)
    out["prologue_a_phase"] = {"mean": {k: round(float(v), 1) for k, v in zip(PRO, pro.mean(0))},
                               "slowest_wg": {k: int(v) for k, v in zip(PRO, pro[slow])}}
    out["ow_setup_cycles"] = float((s[:, 54] - s[:, 53]).mean())  # one-wave mode: stamp 54 ends its setup
    out["l3_setup_split"] = {"54_55": float((s[:, 55] - s[:, 54]).mean()), "pf_store": float((s[:, 56] - s[:, 55]).mean()),
                             "to_barrier_done": float((s[:, 31] - s[:, 56]).mean())}
    out["dma_issue_split"] = {"i_patches": float((s[:, 62] - s[:, 58]).mean()), "level_table": float((s[:, 63] - s[:, 62]).mean()),
                              "j_prefetch": float((s[:, 59] - s[:, 63]).mean())}
    out["prologue_split"] = {"point_load": float((s[:, 58] - s[:, 60]).mean()), "dma_issue": float((s[:, 59] - s[:, 58]).mean()),
                             "dma_wait_barrier": float((s[:, 50] - s[:, 59]).mean())}
    if ovl:  # waves 1-3's overlapped A phase done (slots 49, 39, 29), from the level-3 iteration start
        out["ovl_a_done_after_l3_start"] = {f"wave{k}": round(float((s[:, 59 - 10 * k] - s[:, 31]).mean()), 1)
                                            for k in (1, 2, 3)}
        out["ovl_l3_iters_cycles"] = round(float((s[:, 37] - s[:, 32]).mean()), 1)
    prev_end = s[:, 53]
    for lev in range(3, -1, -1):
        b = lev * 10
        d = np.stack([s[:, b + 1] - prev_end, s[:, b + 2] - s[:, b + 1], s[:, b + 7] - s[:, b + 2]], 1)
        prev_end = s[:, b + 7]
        iters = s[:, b + 8]
        out[f"L{lev}"] = {
            "mean": {k: round(float(v), 1) for k, v in zip(PH, d.mean(0))},
            "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
            "cycles_per_iter": round(float(d[:, 2].sum() / max(iters.sum(), 1)), 1),
            "slowest_wg": {k: int(v) for k, v in zip(PH, d[slow])} | {"iters": int(iters[slow])},
        }
    it = s[:, 40:48]
    n_it = sum(s[:, lev * 10 + 8] for lev in range(4))
    tot_it = n_it.sum()
    out["iteration_phases_cycles_per_iter"] = {
        "products": round(float(it[:, 0].sum() / tot_it), 1), "reduce_barrier": round(float(it[:, 1].sum() / tot_it), 1),
        "chain_combine": round(float(it[:, 2].sum() / tot_it), 1), "solve": round(float(it[:, 3].sum() / tot_it), 1),
        "chain_path_fraction": round(float(it[:, 4].sum() / tot_it), 3), "restage_fraction": round(float(it[:, 5].sum() / tot_it), 3),
        "class_path_fraction": round(float(it[:, 6].sum() / tot_it), 3)}
    t0 = s[:, 60].min()
    ends = (s[:, 61] - t0) / 1e3
    out["wg_end_kcycles_percentiles"] = {str(q): round(float(np.percentile(ends, q)), 1) for q in (10, 50, 90, 99, 100)}
    out["wg_iterations_percentiles"] = {str(q): float(np.percentile(n_it, q)) for q in (10, 50, 90, 99, 100)}
    # per-iteration cost of the slowest workgroups (they run mostly alone in the tail)
    order = np.argsort(tot)[-8:]
    out["slowest8"] = [{"wg_kcycles": round(float(tot[i]) / 1e3, 1), "iters": int(n_it[i]),
                        "iter_cycles": round(float(sum(s[i, l * 10 + 7] - s[i, l * 10 + 2] for l in range(4)) / max(n_it[i], 1)), 1),
                        "chain_frac": round(float(s[i, 44]) / max(n_it[i], 1), 2)} for i in order]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
