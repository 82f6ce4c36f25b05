"""Steady-state window of a rocprofv3 kernel trace of bench.py (profiles/scripts/timeline.sh):
the kernels of a few consecutive sub-batches in the middle of the pipelined run, with their queue."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/tl'}/**/*kernel_trace.csv", recursive=True)[0]
r = list(csv.DictReader(open(f)))
ev = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:16],
             x.get("Queue_Id", "")) for x in r)
sft = [e for e in ev if e[2].startswith("k_sft_nodes")]
mid = len(sft) // 2
t0, t1 = sft[mid][0], sft[mid + 3][0]
print("sub-batch periods (k_sft_nodes starts, us):", [round((sft[i + 1][0] - sft[i][0]) / 1e3, 1) for i in range(mid, mid + 6)])
for s, e, n, q in ev:
    if t0 <= s <= t1:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3s}  {n}")
# busy fraction of each queue over the window (union of its kernels' intervals)
busy = {}
for s, e, n, q in ev:
    if t0 <= s <= t1:
        busy.setdefault(q, []).append((s, min(e, t1)))
for q, iv in sorted(busy.items()):
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print(f"queue {q}: busy {100 * tot / (t1 - t0):.0f} % of the {(t1 - t0) / 1e3:.0f} us window")
