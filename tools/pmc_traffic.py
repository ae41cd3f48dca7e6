#!/usr/bin/env python3
"""Per-kernel HBM-side traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE;
separate passes, MI355X_MICROARCH.md rocprofv3 PMC slots) over the same command.

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch. gfx950 correction, calibrated on this
pool with tools/fetch_calib.hip (profiles/r03a_pmc_calibration.json: 1 GiB streamed per access width):
FETCH_SIZE counts 4-, 8- and 16-B per-lane reads at exactly half their bytes (x2 restores them) and
does not count 2-B per-lane reads at all; WRITE_SIZE is exact for 2-, 4-, 8- and 16-B stores. So
`fetch_bytes_x2` is the fetched bytes of every kernel whose reads are >= 4 B per lane — all of them
except the owner pass, whose 2-B row reads (~0.11 GB per lego step) are missing from its figure, which
is therefore a lower bound. The raw counter is kept as `fetch_kib`.

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if not name.startswith("nerf::") and "nerf::" not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        vals[short].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (None, 0))
        w, nw = write.get(k, (None, 0))
        out[k] = {"fetch_kib": f, "write_kib": w, "launches": max(nf, nw),
                  "fetch_bytes_x2": None if f is None else 2 * 1024 * f,
                  "write_bytes": None if w is None else 1024 * w,
                  "traffic_bytes": None if (f is None or w is None) else 2 * 1024 * f + 1024 * w}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
