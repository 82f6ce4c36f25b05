"""Timeline of one C2 call (one 1241x376 image through orbfe_extract) from a rocprofv3 kernel +
memory-copy trace of profiles/scripts/r5_c2_trace.py: the last latency-schedule call's kernels and
copies, start / end relative to the call's first operation, with the queue of each.
usage: python c2_timeline.py TRACE_DIR [mode index: the trace script's 60-call groups]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    ev = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                       r.get("Queue_Id", "")))
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", ""), ""))
    ev.sort()
    # calls: k_copy0 starts a call; the latency-schedule calls are the first 60
    starts = [e[0] for e in ev if e[2].endswith("k_copy0")]
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    t0, t1 = starts[60 * m + 58], starts[60 * m + 59]  # the 59th call (warm), up to the next call's k_copy0
    # include the H2D copy just before k_copy0
    pre = [e for e in ev if e[0] < t0 and e[2].startswith("copy")]
    base = pre[-1][0] if pre else t0
    for s, e, name, q in ev:
        if base <= s < t1:
            print(f"{(s - base) / 1e3:8.1f} {(e - base) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q {q:>3}  {name}")


if __name__ == "__main__":
    main()
