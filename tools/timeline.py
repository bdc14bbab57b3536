#!/usr/bin/env python3
"""GPU timeline of a rocprofv3 --kernel-trace run (kernel_trace.csv): busy
(union of kernel intervals) vs idle time per frame-set, and the per-kernel
share of the busy time. Usage: tools/timeline.py <kernel_trace.csv> [sets]"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the timed region: the last N pyramid launches mark frame-sets; use the whole trace span
    t0, t1 = ev[0][0], max(e for _, e, _ in ev)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = {}
    for s, e, n in ev:
        k = n.split("(")[0].replace("void ", "")[:60]
        per[k] = per.get(k, 0) + (e - s)
    span = t1 - t0
    print(f"span {span/1e6:.2f} ms, GPU busy (any kernel) {busy/1e6:.2f} ms = {100*busy/span:.1f} %")
    for k, v in sorted(per.items(), key=lambda x: -x[1])[:12]:
        print(f"  {v/1e6:9.2f} ms  {k}")


if __name__ == "__main__":
    main()
