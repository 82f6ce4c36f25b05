"""Mean duration per (kernel, grid) of rocprofv3 kernel-trace CSVs: trace_summary.py DIR..."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not f:
        print(d, "no trace")
        continue
    acc = defaultdict(list)
    for x in csv.DictReader(open(f[0])):
        acc[(x["Kernel_Name"].split("(")[0][:24], x["Grid_Size_X"])].append(
            (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
    print(d)
    for k, v in sorted(acc.items()):
        if len(v) >= 5:
            v = v[3:]
            print(f"   {k[0]:26s} {k[1]:>8s} {sum(v) / len(v):9.1f} us  (n={len(v)})")
