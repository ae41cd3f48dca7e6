#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats kernel_stats.csv into a short markdown table."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main(path, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls | avg us | total ms | % |{' per step ms |' if steps else ''}")
    print(f"|---|---|---|---|---|{'---|' if steps else ''}")
    for r in rows:
        t = float(r["TotalDurationNs"])
        line = f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {t / 1e6:.3f} | {100 * t / tot:.1f} |"
        if steps:
            line += f" {t / 1e6 / steps:.3f} |"
        print(line)
    print(f"\ntotal kernel time {tot / 1e6:.3f} ms" + (f" = {tot / 1e6 / steps:.3f} ms/step" if steps else ""))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
