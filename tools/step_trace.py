#!/usr/bin/env python3
"""The kernel sequence of the last training step in a rocprofv3 --kernel-trace CSV (a bench run): one
line per kernel with its start offset from the step's first kernel, its duration and the idle gap
before it, then the step's span, kernel-busy time and summed gaps. A step starts at each launch of
the first kernel of the iteration (default: rays_pack_kernel).

usage: step_trace.py kernel_trace.csv [FIRST_KERNEL_SUBSTRING]"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)[:70]


def main(path, first="rays_pack_kernel"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(starts) < 2:
        sys.exit(f"fewer than two launches of {first}")
    step = rows[starts[-2]:starts[-1]]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end, busy, gaps = t0, 0, 0
    print("| start us | dur us | gap us | kernel |\n|---|---|---|---|")
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - prev_end)
        print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {gap / 1e3:.1f} | {short(r['Kernel_Name'])} |")
        busy += e - s
        gaps += gap
        prev_end = max(prev_end, e)
    span = int(rows[starts[-1]]["Start_Timestamp"]) - t0
    print(f"\nstep span {span / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us, "
          f"{len(step)} kernels")


if __name__ == "__main__":
    main(*sys.argv[1:])
