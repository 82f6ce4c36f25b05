"""C2 latency A/B of the input path of a host-buffer call: one 1241x376 image through orbfe_extract
with k_copy0 reading the pinned staging buffer's rows over PCIe and the results written straight into
the pinned host mirror (zero copy in + out, the default: zc_rows_out), the same with the staging laid
out as pyramid level 0 by the host and one straight k_copy_l0 (zero copy mode 2: zc_l0_out), zero
copy in only, and H2D / D2H copies
(orbfe_debug_set_zero_copy(h, 0, 0)), all with the default k_pyramid, the copies also with the
per-level chain; interleaved rounds of 200 calls, outputs compared bit for bit.
usage: python profiles/scripts/c2_zero_copy.py [rounds]"""
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
    if os.environ.get("C2_SEQ_IMAGE"):  # the bench's C2 image: frame 0 of its driving sequence
        from orb_slam2_2021_amd.extractor import synth_sequence_frame
        im = synth_sequence_frame(0x0C3, 0, rows, cols)
        img = np.ascontiguousarray(im[0] if isinstance(im, tuple) else im)
    else:
        img = np.ascontiguousarray(synth_frame(3, rows, cols))
    lib = L.lib()
    modes = {"zc_l0_out": (2, 1, True), "zc_rows_out": (1, 1, True), "zc_in": (1, 0, True), "copies": (0, 0, True),
             "copies_chain": (0, 0, False)}
    exts = {}
    for m, (zi, zo, pyr) in modes.items():
        e = ORBextractor(2000, 1.2, 8, 20, 7)
        L.check(L.lib().orbfe_debug_set_zero_copy(e._h, zi, zo), "zero_copy")
        if not pyr:
            e.debug_set_pyramid_tiles((0, 0), (0, 0))
        exts[m] = e
    ref = "copies_chain"
    cap = exts[ref].max_keypoints(rows, cols)
    out = {m: (np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()) for m in modes}

    def call(m):
        k, d, n = out[m]
        L.check(lib.orbfe_extract(exts[m]._h, L.ptr(img), rows, cols, c_size_t(cols), L.ptr(k), cap, L.ptr(d),
                                  byref(n)), "orbfe_extract")

    for m in modes:
        for _ in range(20):
            call(m)
    n0 = out[ref][2].value
    for m in modes:
        n = out[m][2].value
        same = n == n0 and out[m][0][:n].tobytes() == out[ref][0][:n0].tobytes() and \
            np.array_equal(out[m][1][:n], out[ref][1][:n0])
        same_pyr = all(np.array_equal(exts[m].level(l), exts[ref].level(l)) for l in range(8))
        print(f"{m:10s} keypoints {n}  identical: {same}  pyramid identical: {same_pyr}", flush=True)
    res = {m: [] for m in modes}
    for r in range(rounds):
        for m in modes:
            t = []
            for _ in range(200):
                t0 = time.perf_counter()
                call(m)
                t.append(time.perf_counter() - t0)
            res[m] += t
            print(f"round {r} {m:10s} p50 {np.median(t) * 1e3:.4f} ms  min {np.min(t) * 1e3:.4f} ms", flush=True)
    for m in modes:
        t = np.array(res[m])
        print(f"ALL {m:10s} p50 {np.median(t) * 1e3:.4f} ms  p99 {np.percentile(t, 99) * 1e3:.4f} ms  "
              f"min {t.min() * 1e3:.4f} ms")


if __name__ == "__main__":
    main()
