#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs (separate passes) to HBM bytes per
launch per kernel, with the gfx950 corrections of MI355X_MICROARCH.md ("HBM"): FETCH_SIZE (KiB)
counts half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE (KiB) is taken as is.

usage: pmc_summary.py FETCH_CSV WRITE_CSV [OUT_JSON]
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0]
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) & set(write)):
        if k.startswith("__amd"):
            continue
        fb = 2.0 * fetch[k][0] * 1024.0
        wb = write[k][0] * 1024.0
        out[k] = {"fetch_bytes_corrected": round(fb), "write_bytes": round(wb),
                  "traffic_bytes_per_launch": round(fb + wb), "launches": fetch[k][1]}
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
