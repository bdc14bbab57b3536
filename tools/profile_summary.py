#!/usr/bin/env python3
"""One round's profile summary of a bench command, from its rocprofv3 runs
(tools/profile_round.sh): per kernel the kernel-trace stats (launches, mean /
min / max duration), the PMC HBM bytes per launch (FETCH_SIZE / WRITE_SIZE in
separate passes, corrected by the calibration probe as MI355X_MICROARCH.md's
HBM section prescribes: byte-wide accesses -> the read_u8 / write_u8
factors), SQ counters per launch (SQ_INSTS_VALU, SQ_WAVES, SQ_BUSY_CYCLES,
...), the dispatch resources (VGPRs, scratch bytes per lane), and the sha of
the profiled libpsn_lk.so (bench.py checks it against the binary it runs).

usage: profile_summary.py OUTDIR LIB OUT.json
  OUTDIR holds trace/ fetch/ write/ cfetch/ cwrite/ sq/ sq2/ (rocprofv3 -d dirs)
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def counters(d):
    """{kernel: {counter: [per-dispatch values]}, resources}"""
    per = defaultdict(lambda: defaultdict(list))
    res = {}
    for r in rows(d, "*counter_collection.csv"):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        res[k] = {"vgpr": int(float(r.get("VGPR_Count", 0) or 0)), "sgpr": int(float(r.get("SGPR_Count", 0) or 0)),
                  "scratch_bytes_per_lane": int(float(r.get("Scratch_Size", 0) or 0)),
                  "lds_bytes": int(float(r.get("LDS_Block_Size", 0) or 0)),
                  "workgroup": int(float(r.get("Workgroup_Size", 0) or 0))}
    return per, res


def mean(v):
    return sum(v) / len(v) if v else 0.0


def trace_stats(d):
    """Per kernel of a --kernel-trace run: launches, mean / min / max duration and
    busy_us = the union of its launches' execution intervals (launches of one
    kernel that overlap on several streams count once), plus the trace span."""
    iv = defaultdict(list)
    t0, t1 = None, None
    for r in rows(d, "*kernel_trace.csv"):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv[short(r["Kernel_Name"])].append((a, b))
        t0 = a if t0 is None else min(t0, a)
        t1 = b if t1 is None else max(t1, b)
    out = {}
    for k, v in iv.items():
        v.sort()
        busy, ce, cs = 0, None, None
        for a, b in v:
            if ce is None or a > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        busy += ce - cs
        du = [b - a for a, b in v]
        out[k] = {"launches": len(v), "avg_us": round(mean(du) / 1e3, 2), "min_us": round(min(du) / 1e3, 2),
                  "max_us": round(max(du) / 1e3, 2), "busy_us": round(busy / 1e3, 1)}
    return out, (round((t1 - t0) / 1e3, 1) if t0 is not None else 0.0)


def pmc_section(d, sub_fetch, sub_write, sub_sq, ff, wf):
    """PMC HBM bytes per launch (calibrated) and SQ_WAIT_ANY / SQ_WAVE_CYCLES of
    each kernel from one workload's separate --pmc passes."""
    fetch, _ = counters(os.path.join(d, sub_fetch))
    write, _ = counters(os.path.join(d, sub_write))
    sq, res = counters(os.path.join(d, sub_sq))
    out = {}
    for k in set(fetch) | set(write) | set(sq):
        e = {}
        fv, wv = fetch.get(k, {}).get("FETCH_SIZE", []), write.get(k, {}).get("WRITE_SIZE", [])
        if fv or wv:
            e["hbm_bytes_per_launch"] = round(mean(fv) * 1024 * ff + mean(wv) * 1024 * wf)
        for c, v in sq.get(k, {}).items():
            e[c] = round(mean(v), 1)
        if e.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in e:
            e["wait_any_frac"] = round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 4)
        e.update(res.get(k) or {})
        out[k] = e
    return out


def main():
    d, lib, out = sys.argv[1:4]
    gib = float(1 << 30)
    cal = {}
    for sub, cname, pref in (("cfetch", "FETCH_SIZE", "read_"), ("cwrite", "WRITE_SIZE", "write_")):
        per, _ = counters(os.path.join(d, sub))
        for k, cs in per.items():
            v = cs.get(cname)
            if k.startswith(pref) and v and mean(v) > 0:
                cal[k + ("_fetch_factor" if cname == "FETCH_SIZE" else "_write_factor")] = gib / (mean(v) * 1024.0)
    ff, wf = cal.get("read_u8_fetch_factor", 2.0), cal.get("write_u8_write_factor", 1.0)
    fetch, res_f = counters(os.path.join(d, "fetch"))
    write, _ = counters(os.path.join(d, "write"))
    sq, res_s = counters(os.path.join(d, "sq"))
    # the SQ_WAIT_ANY pass, with its own SQ_WAVE_CYCLES (the wait fraction comes from one pass)
    sq2, _ = counters(os.path.join(d, "sq2"))
    for k, cs in sq2.items():
        if "SQ_WAIT_ANY" in cs:
            sq[k]["SQ_WAIT_ANY"] = cs["SQ_WAIT_ANY"]
        if "SQ_WAVE_CYCLES" in cs:
            sq[k]["SQ_WAVE_CYCLES_sq2"] = cs["SQ_WAVE_CYCLES"]
    stats = {}
    for r in rows(os.path.join(d, "trace"), "*kernel_stats.csv"):
        stats[short(r["Name"])] = {"launches": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                                   "min_us": round(float(r["MinNs"]) / 1e3, 2),
                                   "max_us": round(float(r["MaxNs"]) / 1e3, 2),
                                   "share_pct": float(r["Percentage"])}
    kernels = {}
    for k in set(stats) | set(fetch) | set(write) | set(sq):
        e = dict(stats.get(k, {}))
        fv, wv = fetch.get(k, {}).get("FETCH_SIZE", []), write.get(k, {}).get("WRITE_SIZE", [])
        if fv or wv:
            e["fetch_kb_reported"] = round(mean(fv), 1)
            e["write_kb_reported"] = round(mean(wv), 1)
            e["hbm_bytes_per_launch"] = round(mean(fv) * 1024 * ff + mean(wv) * 1024 * wf)
        for c, v in sq.get(k, {}).items():
            e[c] = round(mean(v), 1)
        e.update(res_s.get(k) or res_f.get(k) or {})
        kernels[k] = e
    # the isolated launches (tools/bx_time.py under --kernel-trace: the frame-set's
    # forward and chain-step windows, nothing else on the GPU) and the PETS-like
    # mixed-box leg (bench.py --box-dist pets: kernel trace with busy time, PMC
    # passes)
    extra = {}
    if os.path.isdir(os.path.join(d, "iso")):
        iso, span = trace_stats(os.path.join(d, "iso"))
        meta = {}
        if os.path.exists(os.path.join(d, "iso_time.json")):
            try:
                meta = json.loads(open(os.path.join(d, "iso_time.json")).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                meta = {}
        extra["isolated"] = {"kernels": iso, "trace_span_us": span, "bench": meta.get("isolated", meta),
                             "note": "bench.py --mode isolated: the frame-set's forward and backward LK launches "
                                     "(4 cameras x 512 points) back to back, nothing else on the GPU"}
    if os.path.isdir(os.path.join(d, "pets")):
        pk, span = trace_stats(os.path.join(d, "pets"))
        meta = {}
        if os.path.exists(os.path.join(d, "pets_bench.json")):
            try:
                meta = json.loads(open(os.path.join(d, "pets_bench.json")).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                meta = {}
        pm = pmc_section(d, "pets_fetch", "pets_write", "pets_sq2", ff, wf)
        for k, e in pk.items():
            e.update(pm.get(k, {}))
        extra["mixed_boxes"] = {"kernels": dict(sorted(pk.items(), key=lambda kv: -kv[1]["busy_us"])),
                                "trace_span_us": span,
                                "bench": {k: meta.get(k) for k in ("value", "unit", "ms_per_step", "steps", "warmup",
                                                                   "compute")},
                                "note": "bench.py --box-dist pets under --kernel-trace (the timed frames plus warm-up "
                                        "and measurement frames); busy_us = union of a kernel's launch intervals"}
    if os.path.isdir(os.path.join(d, "k4")):
        kk, span = trace_stats(os.path.join(d, "k4"))
        fetch4, _ = counters(os.path.join(d, "k4_fetch"))
        for k, e in kk.items():
            fv = fetch4.get(k, {}).get("FETCH_SIZE", [])
            if fv:
                e["fetch_bytes_per_launch"] = round(mean(fv) * 1024 * ff)
        meta = {}
        if os.path.exists(os.path.join(d, "k4_bench.json")):
            try:
                meta = json.loads(open(os.path.join(d, "k4_bench.json")).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                meta = {}
        extra["tracker_4k"] = {"kernels": dict(sorted(kk.items(), key=lambda kv: -kv[1]["busy_us"])),
                               "trace_span_us": span,
                               "bench": {k: meta.get(k) for k in ("value", "unit", "ms_per_step", "steps", "warmup")},
                               "note": "bench.py at 3840x2160, 8 cameras x 4096 points, 128x320 boxes under "
                                       "--kernel-trace; fetch_bytes_per_launch from a FETCH_SIZE pass (read_u8 factor)"}
    summary = {"lib_sha16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16],
               "calibration": cal, "kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1].get("share_pct", 0))),
               **extra,
               "notes": "hbm_bytes_per_launch = FETCH_SIZE x read_u8 factor + WRITE_SIZE x write_u8 factor "
                        "(KB x 1024); SQ_* are per-launch means of one --pmc pass"}
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({k: {kk: v.get(kk) for kk in ("launches", "avg_us", "hbm_bytes_per_launch", "SQ_INSTS_VALU",
                                                   "scratch_bytes_per_lane", "vgpr")}
                      for k, v in list(summary["kernels"].items())[:6]}, indent=1))


if __name__ == "__main__":
    main()
