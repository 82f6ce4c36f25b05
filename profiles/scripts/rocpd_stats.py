"""Kernel stats CSV (the columns of rocprofv3 --stats' kernel_stats.csv) from a rocprofv3 rocpd
database, for runs recorded in the default .db output format.
usage: python profiles/scripts/rocpd_stats.py <dir containing *.db> > out.csv"""
import glob
import math
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("""select s.display_name, k.end - k.start from rocpd_kernel_dispatch k
                    join rocpd_info_kernel_symbol s on k.kernel_id = s.id""").fetchall()
by = {}
for name, d in rows:
    by.setdefault(name, []).append(d)
total = sum(d for _, d in rows)
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    n, t = len(ds), sum(ds)
    avg = t / n
    sd = math.sqrt(sum((d - avg) ** 2 for d in ds) / n)
    print(f'"{name}",{n},{t},{avg:.6f},{100 * t / total:.2f},{min(ds)},{max(ds)},{sd:.6f}')
