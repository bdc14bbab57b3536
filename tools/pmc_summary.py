#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs.

usage: pmc_summary.py FETCH_DIR WRITE_DIR CALIB_FETCH_DIR CALIB_WRITE_DIR OUT.json

FETCH_SIZE / WRITE_SIZE are reported in KB (TCC_EA0 requests x 64 B). On
gfx950 they are exact only for calibrated access patterns
(MI355X_MICROARCH.md, HBM), so the calibration probe
(tools/probes/probe_hbm_calib.hip, 1 GiB per kernel) gives the factor
true_bytes / reported_bytes for byte-wide and 16-B-wide reads and writes;
the Tracker2D kernels access HBM byte-wide, so the byte-wide factors apply.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def short(name):
    # the box-window kernel has one instantiation per unit count: keep them apart
    i = name.find("lk_kernel_bx<")
    if i >= 0:
        return name[i:name.index(">", i) + 1]
    for k in ("lk_kernel_st", "lk_kernel_lg", "lk_kernel", "pyramid_kernel", "read_u8", "read_x4", "write_u8",
              "write_x4"):
        if k in name:
            return k
    return name[:60]


def main():
    fdir, wdir, cfdir, cwdir, out = sys.argv[1:6]
    gib = float(1 << 30)
    cf, cw = load(cfdir, "FETCH_SIZE"), load(cwdir, "WRITE_SIZE")
    calib = {}
    for k, v in cf.items():
        if short(k).startswith("read_") and sum(v) > 0:
            calib[short(k) + "_fetch_factor"] = gib / (sum(v) / len(v) * 1024.0)
    for k, v in cw.items():
        if short(k).startswith("write_") and sum(v) > 0:
            calib[short(k) + "_write_factor"] = gib / (sum(v) / len(v) * 1024.0)
    ff = calib.get("read_u8_fetch_factor", 1.0)
    wf = calib.get("write_u8_write_factor", 1.0)
    res = {"calibration": calib, "kernels": {}}
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    for k in set(fetch) | set(write):
        fv, wv = fetch.get(k, []), write.get(k, [])
        fkb = sum(fv) / len(fv) if fv else 0.0
        wkb = sum(wv) / len(wv) if wv else 0.0
        res["kernels"][short(k)] = {
            "dispatches": max(len(fv), len(wv)),
            "fetch_kb_reported": round(fkb, 1), "write_kb_reported": round(wkb, 1),
            "hbm_bytes_per_launch": round(fkb * 1024 * ff + wkb * 1024 * wf),
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
