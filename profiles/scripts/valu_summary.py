"""Per-kernel VALU / SALU wave-instructions per sub-batch from pmc_bench_valu.sh's counter CSV."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcV/run_counter_collection.csv"
sub = int(sys.argv[2]) if len(sys.argv) > 2 else 36  # warmup 16 + probe 4 + steps 16
acc = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(path)):
    acc[row["Kernel_Name"].split("(")[0][:30]][row["Counter_Name"]] += float(row["Counter_Value"])
tot = defaultdict(float)
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"]):
    print(f"{k:32s} VALU/sub {c['SQ_INSTS_VALU'] / sub / 1e6:7.2f}M  SALU/sub {c['SQ_INSTS_SALU'] / sub / 1e6:6.2f}M")
    for x in c:
        tot[x] += c[x]
print(f"total VALU/sub {tot['SQ_INSTS_VALU'] / sub / 1e6:.1f}M  SALU/sub {tot['SQ_INSTS_SALU'] / sub / 1e6:.1f}M")
