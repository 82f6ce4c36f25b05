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
usage: pmc_waits.py CSV [kernel-prefix ...] [--json OUT.json --workload JSON]
--json also writes the per-kernel figures (per launch: SQ_INSTS_VALU, the wave-time split, waves per
SIMD, the PMC run's kernel time and effective clock) for bench.py's issue-side roofline."""
import csv
import json
import sys
from collections import defaultdict

args = sys.argv[1:]
json_out = workload = None
if "--json" in args:
    i = args.index("--json")
    json_out = args[i + 1]
    del args[i:i + 2]
if "--workload" in args:
    i = args.index("--workload")
    workload = json.loads(args[i + 1])
    del args[i:i + 2]
sys.argv = [sys.argv[0]] + args

acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        c = acc[k][row["Counter_Name"]]
        c[0] += float(row["Counter_Value"])
        c[1] += 1
want = sys.argv[2:]
doc = {"source": "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE (one pass) of " + sys.argv[1]
                  + "; per-dispatch means; profiles/pmc_waits.py",
       "workload": workload, "kernels": {}}
print(f"{'kernel':26s} {'us/launch':>9s} {'active':>7s} {'w_inst':>7s} {'w_any':>7s} {'waves/SIMD':>10s} {'VALU busy':>9s}")
for k in sorted(acc):
    if want and not any(k.startswith(w) for w in want):
        continue
    m = {c: s / n for c, (s, n) in acc[k].items()}
    wc = m.get("SQ_WAVE_CYCLES", 0.0)
    if not wc or "GRBM_GUI_ACTIVE" not in m:
        continue
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    name = k.replace("void ", "").split("<")[0]
    doc["kernels"][name] = {"insts_valu_per_launch": m["SQ_INSTS_VALU"], "active": m["SQ_ACTIVE_INST_ANY"] / wc,
                            "wait_inst": m["SQ_WAIT_INST_ANY"] / wc, "wait_any": m["SQ_WAIT_ANY"] / wc,
                            "waves_per_simd": wc * 4 / (cyc * 1024), "us_per_launch_at_2p4GHz": cyc / 2400,
                            "valu_busy": m["SQ_INSTS_VALU"] * 2 / (cyc * 1024)}
    print(f"{k:26s} {cyc / 2400:9.1f} {m['SQ_ACTIVE_INST_ANY'] / wc:7.1%} {m['SQ_WAIT_INST_ANY'] / wc:7.1%} "
          f"{m['SQ_WAIT_ANY'] / wc:7.1%} {wc * 4 / (cyc * 1024):10.2f} {m['SQ_INSTS_VALU'] * 2 / (cyc * 1024):9.1%}")
if json_out:
    with open(json_out, "w") as f:
        json.dump(doc, f, indent=1)
