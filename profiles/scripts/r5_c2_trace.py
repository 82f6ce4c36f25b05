"""One 1241x376 image through orbfe_extract, 60 calls per schedule (latency k = 1, then the
throughput schedule; latency k = 1), for a rocprofv3 kernel / memory-copy trace of the C2 call's timeline.
With arguments tx,ty ...: latency k = 1 with k_pyramid at each tiling instead (0,0: the chain).
usage: rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 profiles/scripts/r5_c2_trace.py [tx,ty ...]"""
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
    rows, cols = 376, 1241
    if os.environ.get("C2_SEQ_IMAGE"):  # the bench's C2 image: frame 0 of its driving sequence
        from orb_slam2_2021_amd.extractor import synth_sequence_frame
        im = synth_sequence_frame(0x0C3, 0, rows, cols)
        img = np.ascontiguousarray(im[0] if isinstance(im, tuple) else im)
    else:
        img = np.ascontiguousarray(synth_frame(3, rows, cols))
    lib = L.lib()
    tilings = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
    modes = [(1, t) for t in tilings] if tilings else [(1, None), (0, None)]
    for k, t in modes:
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        e.debug_set_latency_schedule(k)
        if t is not None:
            e.debug_set_pyramid_tiles(t, (0, 0))
        cap = e.max_keypoints(rows, cols)
        kp, d, n = np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()
        for i in range(60):
            t0 = time.perf_counter()
            L.check(lib.orbfe_extract(e._h, L.ptr(img), rows, cols, c_size_t(cols), L.ptr(kp), cap, L.ptr(d),
                                      byref(n)), "orbfe_extract")
            if i == 59:
                print(f"k={k} tiles={t} last call {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
        time.sleep(0.05)  # a gap in the trace between the schedules


if __name__ == "__main__":
    main()
