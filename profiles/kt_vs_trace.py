#!/usr/bin/env python3
"""The bench line's kernel times (orbfe_ktimer: dispatch-bound events less the calibrated timer
overhead) against rocprofv3's kernel trace of the same run, kernel by kernel.

usage: kt_vs_trace.py TRACE_CSV BENCH_LOG [OUT]
TRACE_CSV: rocprofv3 --kernel-trace output (run_kernel_trace.csv) of `bench.py ARGS`;
BENCH_LOG: that run's stdout (its JSON line). The timed region is located in the trace as the
steps x batches_per_step sub-batches (one k_describe each, in enqueue order) that end at the
largest idle gap of the run (the oracle parity check after the timed region); the event
sub-batches are every event_every-th group of len(handles) sub-batches from its start, as bench.py
selects them. Prints, per kernel: the trace's mean duration over the whole run, over the timed
region and over its event sub-batches, and the line's per-launch time."""
import collections
import csv
import json
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].replace("(anonymous namespace)::", "")


def main():
    trace, log = sys.argv[1], sys.argv[2]
    line = next(json.loads(l) for l in open(log) if l.startswith("{"))
    steps = line["steps"]
    per_step = line["config"]["subbatches_per_step"]
    handles = line["config"].get("extractor_handles", 4)
    every = line["config"].get("event_every", 8)
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        by[short(r["Kernel_Name"])].append((int(r["Correlation_Id"]), int(r["Start_Timestamp"]),
                                            int(r["End_Timestamp"])))
    desc = sorted(by["k_describe"])
    gaps = [(desc[i][1] - desc[i - 1][2], i) for i in range(1, len(desc))]
    end = max(gaps)[1]  # first sub-batch after the parity check's gap
    start = end - steps * per_step
    n_sub = len(desc)
    out = {"timed_region_subbatches": [start, end], "event_every": every, "handles": handles, "kernels": {}}
    kus = line.get("kernels_us_per_subbatch", {})
    print(f"timed region: sub-batches {start}..{end} of {n_sub}; events on every {every}th group of {handles}")
    print(f"{'kernel':18s} {'launches/sb':>11s} {'trace run':>10s} {'trace timed':>11s} {'trace event sb':>14s} {'line':>8s}")
    for k, v in sorted(by.items(), key=lambda kv: -sum(e - s for _, s, e in kv[1])):
        v = sorted(v)
        if len(v) % n_sub:  # launches not one-per-sub-batch-multiple (matching-side kernels skip some)
            continue
        per = len(v) // n_sub
        d = [(e - s) / 1e3 for _, s, e in v]
        timed = d[start * per:end * per]
        ev = [x for i, x in enumerate(timed) if ((i // per) // handles) % every == 0]
        line_us = kus.get(k, 0.0) / per if k in kus else None
        row = {"launches_per_subbatch": per, "trace_run_us": sum(d) / len(d), "trace_timed_us": sum(timed) / len(timed),
               "trace_event_subbatches_us": sum(ev) / len(ev), "line_us": line_us}
        out["kernels"][k] = {a: (round(b, 2) if isinstance(b, float) else b) for a, b in row.items()}
        print(f"{k:18s} {per:11d} {row['trace_run_us']:10.1f} {row['trace_timed_us']:11.1f} "
              f"{row['trace_event_subbatches_us']:14.1f} {line_us if line_us is None else round(line_us, 1)!s:>8s}")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
