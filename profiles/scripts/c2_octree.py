"""C2 (one 1241x376 image through orbfe_extract, host buffers in and out: what
ORBextractor::operator() costs a caller) with DistributeOctTree's small-call block at 256 / 512 /
1024 threads (orbfe_debug_set_octree_threads), interleaved rounds, p50 / p10 per setting; then the
octree launches' device time per call (orbfe_ktimer, dispatch-bound events) for each setting.
usage: python c2_octree.py [rounds] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from orb_slam2_2021_amd import ORBextractor, synth_frame  # noqa: E402
from orb_slam2_2021_amd import _lib as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    img = synth_frame(0, 376, 1241)
    settings = (256, 512, 1024)
    exts = {}
    for t in settings:
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        e.debug_set_octree_threads(t, 256)
        for _ in range(20):
            e(img)
        exts[t] = e
    res = {t: [] for t in settings}
    for r in range(rounds):
        for t in settings:
            e = exts[t]
            xs = []
            for _ in range(reps):
                t0 = time.perf_counter()
                e(img)
                xs.append(time.perf_counter() - t0)
            res[t] += xs
            print(f"round {r} threads {t:4d}: p50 {np.median(xs) * 1e3:.4f} ms", flush=True)
    for t in settings:
        a = np.array(res[t]) * 1e3
        print(f"threads {t:4d}: p50 {np.median(a):.4f} ms  p10 {np.percentile(a, 10):.4f}  p90 {np.percentile(a, 90):.4f}"
              f"  (n={len(a)})")
    # device time of the octree launches per call (every kernel timed by its dispatch events)
    ov = L.ktimer_calibrate(0)
    for t in settings:
        L.ktimer_reset()
        L.ktimer_select(True)
        for _ in range(100):
            exts[t](img)
        L.ktimer_select(False)
        kt = L.ktimer_read()
        ms, cnt = kt.get("k_octree", (0.0, 0))
        per_call = (ms - cnt * ov * 1e-3) / 100 * 1e3
        print(f"threads {t:4d}: k_octree {per_call:.1f} us per call ({cnt / 100:.0f} launches), "
              f"all kernels {sum(v[0] for v in kt.values()) / 100 * 1e3:.1f} us summed")


if __name__ == "__main__":
    main()
