"""Per-kernel VALU / SALU wave-instructions per sub-batch from a bench.py counter CSV (pmc_bench_valu.sh,
or refresh_profiles.sh's pmcWait pass, which has no SALU counter)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcV/run_counter_collection.csv"
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for row in csv.DictReader(open(path)):
    k = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:30]
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    disp[k].add(row["Dispatch_Id"])
sub = len(disp["k_sft_finish"])  # one per C3 sub-batch
ext = len(disp["k_describe"])  # one per 64-image extraction (the bench's setup adds a few)
EXTRACT = ("k_fast", "void k_fast", "k_resize", "k_blur", "k_describe", "k_octree", "k_copy0", "k_pyramid")
print(f"{sub} sub-batches (k_sft_finish dispatches), {ext} extractions (k_describe dispatches); extraction "
      "kernels per extraction, the others per sub-batch")
tot = defaultdict(float)
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"]):
    d = ext if k.startswith(EXTRACT) else sub
    if d == 0:
        continue
    print(f"{k:32s} VALU {c['SQ_INSTS_VALU'] / d / 1e6:7.2f}M  SALU {c.get('SQ_INSTS_SALU', 0.0) / d / 1e6:6.2f}M")
    for x in c:
        tot[x] += c[x] / d
print(f"total per sub-batch: VALU {tot['SQ_INSTS_VALU'] / 1e6:.1f}M  SALU {tot.get('SQ_INSTS_SALU', 0.0) / 1e6:.1f}M")
