"""C2 latency A/B: one 1241x376 image through orbfe_extract (host buffers in and out, the bench's
c2_latency call) with the throughput schedule (k = 0) and the latency schedule
(orbfe_debug_set_latency_schedule(k): FAST + DistributeOctTree of levels 0..k-1 on the side stream),
interleaved rounds of 200 calls; also the stereo pair in one call. Outputs compared bit for bit.
usage: python profiles/scripts/r5_c2_sched.py [rounds]"""
import os
import sys
import time
from ctypes import byref, c_int, c_size_t

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from orb_slam2_2021_amd import ORBextractor, synth_frame  # noqa: E402
from orb_slam2_2021_amd import _lib as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rows, cols = 376, 1241
    img = np.ascontiguousarray(synth_frame(3, rows, cols))
    lib = L.lib()
    # latency schedule k (0: off). (Round 5 also measured a build that enqueued the side's work
    # after the main chain's, "d" in profiles/r5_c2_sched.txt: removed.)
    modes = {"thru": 0, "lat_k1": 1, "lat_k2": 2, "lat_k3": 3}
    exts = {}
    for m, k in modes.items():
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        e.debug_set_latency_schedule(k)
        exts[m] = e
    cap = exts["thru"].max_keypoints(rows, cols)
    out = {m: (np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()) for m in modes}

    def call(m):
        k, d, n = out[m]
        L.check(lib.orbfe_extract(exts[m]._h, L.ptr(img), rows, cols, c_size_t(cols), L.ptr(k), cap, L.ptr(d),
                                  byref(n)), "orbfe_extract")

    for m in modes:
        for _ in range(20):
            call(m)
    n0 = out["thru"][2].value
    for m in modes:
        n = out[m][2].value
        same = n == n0 and out[m][0][:n].tobytes() == out["thru"][0][:n0].tobytes() and \
            np.array_equal(out[m][1][:n], out["thru"][1][:n0])
        print(f"{m:8s} keypoints {n}  identical to thru: {same}")
    res = {m: [] for m in modes}
    for r in range(rounds):
        for m in modes:
            t = []
            for _ in range(200):
                t0 = time.perf_counter()
                call(m)
                t.append(time.perf_counter() - t0)
            res[m] += t
            print(f"round {r} {m:8s} p50 {np.median(t) * 1e3:.4f} ms  min {np.min(t) * 1e3:.4f} ms", flush=True)
    for m in modes:
        t = np.array(res[m])
        print(f"ALL {m:8s} p50 {np.median(t) * 1e3:.4f} ms  p99 {np.percentile(t, 99) * 1e3:.4f} ms  "
              f"min {t.min() * 1e3:.4f} ms")


if __name__ == "__main__":
    main()
