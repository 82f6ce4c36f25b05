#!/usr/bin/env python3
"""Per-kernel mean of every counter in a rocprofv3 --pmc counter_collection CSV.
usage: pmc_kernel.py CSV [kernel-prefix ...]"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        c = acc[k][row["Counter_Name"]]
        c[0] += float(row["Counter_Value"])
        c[1] += 1
want = sys.argv[2:]
for k in sorted(acc):
    if want and not any(k.startswith(w) for w in want):
        continue
    print(k)
    for c, (s, n) in sorted(acc[k].items()):
        print(f"  {c:28s} {s / n:16.1f}  (n={n})")
