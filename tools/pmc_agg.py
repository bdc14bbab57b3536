#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter_collection.csv (millions per launch)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
ids = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    ids[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    n = len(ids[k])
    print(k, n, {c: round(x / n / 1e6, 3) for c, x in sorted(v.items())})
