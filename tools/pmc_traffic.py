#!/usr/bin/env python3
"""Per-kernel HBM-side traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE;
separate passes, MI355X_MICROARCH.md rocprofv3 PMC slots) over the same command.

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch. gfx950 correction, calibrated on this
pool with tools/fetch_calib.hip (profiles/r03a_pmc_calibration.json: 1 GiB streamed per access width):
FETCH_SIZE counts 4-, 8- and 16-B per-lane reads at exactly half their bytes (x2 restores them) and
does not count 2-B per-lane reads at all; WRITE_SIZE is exact for 2-, 4-, 8- and 16-B stores. So
`fetch_bytes` is FETCH_SIZE x 2 for every kernel whose reads are >= 4 B per lane, and for the owner pass
(its entries: an 8-B value and a 2-B row each) FETCH_SIZE / 0.642, the ratio the calibration measured
on exactly that access pattern (`owner_pattern_fetch_over_entry_bytes`; x2 would overstate it by about
0.2 GB per lego step). The raw counter is kept as `fetch_kib`, the factor as `fetch_factor`.

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json
"""
import collections
import csv
import json
import os
import sys

CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                     "r03a_pmc_calibration.json")


def fetch_factor(kernel):
    """Bytes per FETCH_SIZE byte for this kernel's access pattern (the calibration file)."""
    c = json.load(open(CALIB))
    if "hash_bwd_owner_kernel" in kernel:
        return 1.0 / c["owner_pattern_fetch_over_entry_bytes"]
    return 1.0 / c["read_8B_fetch_over_bytes"]


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
        ff = fetch_factor(k)
        out[k] = {"fetch_kib": f, "write_kib": w, "launches": max(nf, nw), "fetch_factor": round(ff, 4),
                  "fetch_bytes": None if f is None else ff * 1024 * f,
                  "write_bytes": None if w is None else 1024 * w,
                  "traffic_bytes": None if (f is None or w is None) else ff * 1024 * f + 1024 * w}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
