#!/usr/bin/env python3
"""HBM bytes of one C5 search (isInFrustum + SearchByProjection kernels of orbfe_search_local_points)
from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of profiles/scripts/c5_only.py, with the
gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE doubled). Per search = sum over the call's
kernels of (mean per launch x launches per search). usage: pmc_c5_summary.py FETCH WRITE SEARCHES [OUT]"""
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
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0]
            acc[k][0] += float(row["Counter_Value"])
            acc[k][1] += 1
    return acc


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    searches = int(sys.argv[3])
    kernels, total = {}, 0.0
    for k in sorted(set(fetch) & set(write)):
        if not (k.startswith("k_frustum") or k.startswith("k_sbp") or k.startswith("k_grid")):
            continue
        # the totals over all launches of the run / searches (every search launches the same set)
        b = (2.0 * fetch[k][0] + write[k][0]) * 1024.0 / searches
        kernels[k] = {"traffic_bytes_per_search": round(b), "launches": fetch[k][1]}
        total += b
    doc = {"workload": {"map_points": 50000, "frames": "640x480 synthetic, bench.c5_scene"},
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of profiles/scripts/c5_only.py; "
                     "FETCH_SIZE x 2 (gfx950 correction), KiB -> bytes; summed over the search's kernels",
           "traffic_bytes_per_search": round(total), "kernels": kernels}
    text = json.dumps(doc, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
