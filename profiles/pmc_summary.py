#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs (separate passes) to HBM bytes per
launch per kernel, with the gfx950 corrections of MI355X_MICROARCH.md ("HBM"): FETCH_SIZE (KiB)
counts half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE (KiB) is taken as is.

usage: pmc_summary.py FETCH_CSV WRITE_CSV [OUT_JSON]
Per sub-batch (one C3 batch of 64 images; bench.py's `traffic_bytes_per_step` key keeps its
round-1 name) = mean per launch x launches per sub-batch (k_resize_win: one per pyramid level;
k_fast: levels 0..K-1 each beside the resize chain + the rest; every other kernel once), counted as
each kernel's launches over k_describe's.
"""
import csv
import json
import sys
from collections import defaultdict


def kname(raw):
    name = raw.replace("(anonymous namespace)::", "").split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    return name.split("<")[0]


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = kname(row["Kernel_Name"])
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    # launches per sub-batch: each kernel's launch count over k_describe's (one per sub-batch)
    ref = fetch.get("k_describe", (0, 0))[1]
    lps = {k: max(1, round(c / ref)) for k, (_, c) in fetch.items()} if ref else {}
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        if k.startswith("__amd") or k.startswith("at::") or "native" in k:
            continue
        fb = 2.0 * fetch[k][0] * 1024.0
        wb = write[k][0] * 1024.0
        per_step = lps.get(k, 1)
        kernels[k] = {"fetch_bytes_corrected_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                      "traffic_bytes_per_launch": round(fb + wb), "launches_per_step": per_step,
                      "traffic_bytes_per_step": round((fb + wb) * per_step)}
    doc = {"workload": {"cols": 1241, "rows": 376, "batch": 32, "pairs": "kf", "stereo": True},
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     "bench.py --no-cpu --no-legs (profiles/scripts/refresh_profiles.sh; default workload: KeyFrame "
                     "pairs, ComputeStereoMatches on); FETCH_SIZE x 2 (gfx950 correction), KiB -> bytes; per launch "
                     "and per sub-batch of 64 images",
           "kernels": kernels}
    text = json.dumps(doc, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
