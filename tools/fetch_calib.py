#!/usr/bin/env python3
"""Counter bytes / true bytes per access width from tools/fetch_calib.hip's two PMC passes (the
second launch of each kernel; the first can carry one-time costs).

usage: fetch_calib.py FETCH_counter_collection.csv WRITE_counter_collection.csv calib.json
"""
import collections
import csv
import json
import sys


def per_dispatch(path, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(1024.0 * float(r["Counter_Value"]))
    return out


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    info = json.load(open(sys.argv[3]))
    n = info["stream_bytes"]
    res = {"stream_bytes": n}
    width = {"unsigned short": 2, "unsigned int": 4, "unsigned long": 8, "uint4": 16, "HIP_vector_type<unsigned int, 4u>": 16}
    for name, vals in fetch.items():
        if name.startswith("stream_read"):
            t = name[name.index("<") + 1:name.rindex(">")]
            res[f"read_{width.get(t, t)}B_fetch_over_bytes"] = vals[-1] / n
        elif name.startswith("owner_pattern"):
            res["owner_pattern_fetch_bytes"] = vals[-1]
            res["owner_pattern_entry_bytes"] = info["owner_entry_bytes"]
            res["owner_pattern_fetch_over_entry_bytes"] = vals[-1] / info["owner_entry_bytes"]
            res["owner_pattern_lines_128B_bytes"] = 128 * info["owner_lines_touched_128"]
    for name, vals in write.items():
        if name.startswith("stream_write"):
            t = name[name.index("<") + 1:name.rindex(">")]
            res[f"write_{width.get(t, t)}B_write_over_bytes"] = vals[-1] / n
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
