"""BASELINE config C5's device part alone, for rocprofv3 passes: SearchLocalPoints (isInFrustum +
SearchByProjection th=3, Tracking.cc:1186-1213) of the bench's 16 frames against its 50k-MapPoint
local map, repeated. python profiles/scripts/c5_only.py [reps] [--per-kernel] (--per-kernel: every
kernel's dispatch-bound device time per search, orbfe_ktimer; --resident: the map in HBM)"""
import os
import sys
import time
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from orb_slam2_2021_amd import ORBmatcher  # noqa: E402
from orb_slam2_2021_amd import _lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ext, F0, G, imgs, poses, _ = bench.c5_scene(2000, 1, 0, None)
    frames = [bench.c5_frame(ext, img, tcw) for img, tcw in zip(imgs, poses)]
    if "--resident" in sys.argv:
        import torch
        from orb_slam2_2021_amd.frames import DeviceMapPointGeometry
        G = DeviceMapPointGeometry(G, device=torch.device("cuda", 0))
    m = ORBmatcher(0.8, True)
    m.SearchLocalPoints(frames[0], G, 3.0)
    m.set_profiling(True)
    if "--per-kernel" in sys.argv:
        L.ktimer_reset()
        L.ktimer_select(True)
    dev, rounds_all = [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        for F in frames:
            m.SearchLocalPoints(F, G, 3.0)
            dev.append(m.last_device_ms())
            rounds_all.append(m.last_stats()[0])
    dt = (time.perf_counter() - t0) / (reps * len(frames))
    n = reps * len(frames)
    rounds = m.last_stats()[0]
    st = np.zeros(16, np.int32)
    L.check(L.lib().orbfe_debug_matcher_sweep_stats(m._h, L.ptr(st)), "sweep_stats")
    print(f"c5: {len(G.flags)} MapPoints, {np.mean([F.N for F in frames]):.0f} keypoints per frame, "
          f"{1e3 * dt:.3f} ms per search (host buffers), device {1e3 * np.mean(dev):.1f} us per search "
          f"(median {1e3 * np.median(dev):.1f}), {reps * len(frames)} searches; sweep (last search): chunks {st[0]}, "
          f"rounds {st[1]}, live queries {st[2]}, sequential chunks {st[3]}, deepest chunk {st[4]} rounds; "
          f"ticks (10 ns) compaction / staging / rounds / commits {st[5]} / {st[6]} / {st[7]} / {st[8]}; "
          f"past the cache {st[9]}; kernel: {st[10]} k shader cycles in {st[11]} ticks = {st[10] * 1e5 / max(st[11], 1):.0f} MHz")
    print("rounds per search:", dict(sorted(Counter(rounds_all).items())))
    if "--per-kernel" in sys.argv:
        L.ktimer_select(False)
        for k, (ms, c) in sorted(L.ktimer_read().items(), key=lambda kv: -kv[1][0]):
            print(f"  {k:22s} {1e3 * ms / n:8.1f} us/search  {c / n:5.1f} launches/search")


if __name__ == "__main__":
    main()
