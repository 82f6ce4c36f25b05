"""Per-call timeline of the first 60 single-image calls of a fresh handle with two streams forced
(autotune off) after K idle extractor handles: does the shared-queue penalty show from the first
call, or develop? usage: python profiles/scripts/c2_queues3.py K"""
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


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    img = np.ascontiguousarray(synth_frame(3, 376, 1241))
    keep = []
    for _ in range(k):
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        e(img)
        keep += [e, torch.cuda.Stream()]
    for rep in range(3):
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        e.debug_set_schedule_autotune(False)
        lib = L.lib()
        cap = e.max_keypoints(376, 1241)
        kp, d, c = np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()
        t = []
        for i in range(60):
            t0 = time.perf_counter()
            L.check(lib.orbfe_extract(e._h, L.ptr(img), 376, 1241, c_size_t(1241), L.ptr(kp), cap, L.ptr(d), byref(c)), "x")
            t.append((time.perf_counter() - t0) * 1e6)
        print(f"handle {rep}: " + " ".join(f"{v:.0f}" for v in t), flush=True)
        keep.append(e)


if __name__ == "__main__":
    main()
