#!/usr/bin/env python3
"""Wave-time breakdown per kernel from a rocprofv3 --pmc CSV holding SQ_WAVE_CYCLES,
SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY (disjoint: they sum to SQ_WAVE_CYCLES,
MI355X_MICROARCH.md 'rocprofv3 PMC slots'), SQ_INSTS_VALU and GRBM_GUI_ACTIVE.
  active     = cycles a wave issued an instruction
  wait_inst  = ready but not issued (dependency / pipe / arbitration stalls)
  wait_any   = parked on s_waitcnt or a barrier (memory and LDS latency)
  waves/SIMD = SQ_WAVE_CYCLES (quad-cycles) * 4 / (kernel cycles * 1024 SIMDs), with kernel cycles =
               GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs: k_describe's 1.41M / 8 = 73 us at
               2.4 GHz, its rocprof duration alone)
  VALU busy  = SQ_INSTS_VALU * 2 cycles (wave64 on SIMD-32) / (kernel cycles * 1024)
usage: pmc_waits.py CSV [kernel-prefix ...]"""
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
print(f"{'kernel':26s} {'us/launch':>9s} {'active':>7s} {'w_inst':>7s} {'w_any':>7s} {'waves/SIMD':>10s} {'VALU busy':>9s}")
for k in sorted(acc):
    if want and not any(k.startswith(w) for w in want):
        continue
    m = {c: s / n for c, (s, n) in acc[k].items()}
    wc = m.get("SQ_WAVE_CYCLES", 0.0)
    if not wc or "GRBM_GUI_ACTIVE" not in m:
        continue
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    print(f"{k:26s} {cyc / 2400:9.1f} {m['SQ_ACTIVE_INST_ANY'] / wc:7.1%} {m['SQ_WAIT_INST_ANY'] / wc:7.1%} "
          f"{m['SQ_WAIT_ANY'] / wc:7.1%} {wc * 4 / (cyc * 1024):10.2f} {m['SQ_INSTS_VALU'] * 2 / (cyc * 1024):9.1%}")
