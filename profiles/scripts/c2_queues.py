"""Does the number of streams a process holds move C2? One 1241x376 image through orbfe_extract
(p50 of 300 calls) on a fresh handle, then again after creating K idle extractor handles (two
streams each) and K torch streams -- the bench measures C2 inside a process that holds the C3
pipeline's streams; GPU_MAX_HW_QUEUES bounds the hardware queues the streams share.
usage: python profiles/scripts/c2_queues.py [K ...]"""
import os
import sys
import time
from ctypes import byref, c_int, c_size_t

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from orb_slam2_2021_amd import ORBextractor, synth_frame  # noqa: E402
from orb_slam2_2021_amd import _lib as L  # noqa: E402


def p50(e, img, n=300):
    lib = L.lib()
    rows, cols = img.shape
    cap = e.max_keypoints(rows, cols)
    k, d, c = np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()
    t = []
    for i in range(n + 20):
        t0 = time.perf_counter()
        L.check(lib.orbfe_extract(e._h, L.ptr(img), rows, cols, c_size_t(cols), L.ptr(k), cap, L.ptr(d), byref(c)), "x")
        t.append(time.perf_counter() - t0)
    return np.median(t[20:]) * 1e3


def fresh(mode):
    e = ORBextractor(2000, 1.2, 8, 20, 7)
    if mode == "inline_side":
        e.debug_set_inline_side(True)
    elif mode == "throughput":
        e.debug_set_latency_schedule(0)
    elif mode == "two_streams":
        e.debug_set_schedule_autotune(False)
    return e


def main():
    ks = [int(a) for a in sys.argv[1:]] or [4, 12]
    img = np.ascontiguousarray(synth_frame(3, 376, 1241))
    keep = []
    modes = ("default", "two_streams", "inline_side")
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}  run_idle={os.environ.get('RUN_IDLE', '1')}")
    for m in modes:
        print(f"idle handles 0 {m:12s}: p50 {p50(fresh(m), img):.4f} ms", flush=True)
    have = 0
    for k in ks:
        while have < k:
            e = ORBextractor(2000, 1.2, 8, 20, 7)
            if os.environ.get("RUN_IDLE", "1") == "1":
                e(img)
            keep.append(e)
            keep.append(torch.cuda.Stream())
            have += 1
        for m in modes:
            e = fresh(m)
            t = p50(e, img)
            extra = ""
            if m == "default":  # the same handle (same queues) with two streams forced
                choice = e.debug_schedule_choice(1)
                e.debug_set_schedule_autotune(False)
                extra = f"  (autotune choice {choice}; this handle with two streams forced: {p50(e, img):.4f} ms)"
            print(f"idle handles {k} {m:12s}: p50 {t:.4f} ms{extra}", flush=True)


if __name__ == "__main__":
    main()
