#!/usr/bin/env python3
"""Summary of a tools/iter_check.sh result directory: python tools/iter_show.py <dir>"""
import json
import sys

d = sys.argv[1]
print(open(f"{d}/tests.log").read().strip().splitlines()[-1])
for f in ("st64", "st160"):
    s = json.load(open(f"{d}/{f}.json"))
    print(f, round(s["wg_cycles_mean"]), s["iterations_mean"], s["serial_b_fraction"])
    print("  ", s["mean"])
    print("  ", s["per_iteration"])
    print("  ", s["serial_b_per_tile_chain_lane_view"])
b = json.loads(open(f"{d}/bench.json").read().strip().splitlines()[-1])
print("bench", b["value"], b["unit"], b["ms_per_step"], "ms/step")
