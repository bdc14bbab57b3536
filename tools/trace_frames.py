#!/usr/bin/env python3
"""Steady-state kernel timeline of a traced Tracker2D bench (rocprofv3
--kernel-trace csv): the kernels of a few frame-sets relative to a forward
launch, with their queue, to read the critical path and the GPU's idle gaps.
  python tools/trace_frames.py gpurun_out/t2/trace/run_kernel_trace.csv [first_set] [nsets]"""
import csv
import sys


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    nsets = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "").replace("psn::", "")
                 .replace("(anonymous namespace)::", "")[:24], r["Queue_Id"]) for r in rows)
    fw = [i for i, e in enumerate(ev) if "bx<10" in e[2]]
    i0, i1 = fw[first], fw[first + nsets]
    t0 = ev[i0][0]
    for s, e, n, q in ev[i0 - 12:i1]:
        print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  q{q} {n}")
    per = (ev[fw[-2]][0] - ev[fw[2]][0]) / (len(fw) - 4) / 1000
    print(f"frame-set period (forward launch to forward launch): {per:.1f} us")


if __name__ == "__main__":
    main()
