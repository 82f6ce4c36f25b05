"""Host-boundary sweep: orbfe_extract_batch wall time on 64 KITTI-shaped host images (run with
ORBFE_HOST_CHUNK set per process)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np

from orb_slam2_2021_amd import ORBextractor, synth_frame
from orb_slam2_2021_amd import _lib as L

n, rows, cols = 64, 376, 1241
host = np.stack([synth_frame(i, rows, cols) for i in range(n)])
ext = ORBextractor(2000, 1.2, 8, 20, 7)
lib = L.lib()
cap = ext.max_keypoints(rows, cols)
kps = np.empty(n * cap, L.KEYPOINT_DTYPE)
desc = np.empty((n * cap, 32), np.uint8)
counts = np.zeros(n, np.int32)
arr = (ctypes.c_void_p * n)(*[host[i].ctypes.data for i in range(n)])
def call():
    L.check(lib.orbfe_extract_batch(ext._h, n, ctypes.cast(arr, ctypes.c_void_p), rows, cols, ctypes.c_size_t(cols),
                                    L.ptr(kps), L.ptr(desc), cap, L.ptr(counts)), "batch")
for _ in range(3):
    call()
ts = []
for _ in range(20):
    t0 = time.perf_counter(); call(); ts.append(time.perf_counter() - t0)
print(f"chunk={os.environ.get('ORBFE_HOST_CHUNK')} p50 {1e3*np.median(ts):.3f} ms  min {1e3*min(ts):.3f} ms  -> {n/2/np.median(ts):.0f} stereo frames/s")
