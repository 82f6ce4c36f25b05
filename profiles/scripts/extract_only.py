"""Extraction only, C3 shape (64 images of 1241x376 per call), for PMC passes on the extractor
kernels: python profiles/scripts/extract_only.py [calls] [--per-kernel] [--side=K]
[--seq] (--seq: the bench's driving-sequence frames instead of orbfe_synth_frame)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from orb_slam2_2021_amd import ORBextractor, synth_frame, synth_sequence_frame
from orb_slam2_2021_amd import _lib as L


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
    B, H, W = 32, 376, 1241
    host = np.zeros((2 * B, H, W), np.uint8)
    for i in range(B):
        if "--seq" in sys.argv:
            l, r = synth_sequence_frame(0x0C3, i, H, W, right=True)
        else:
            l, r = synth_frame(i, H, W, right=True)
        host[i], host[B + i] = l, r
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(host).to(dev)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, device=0)
    for a in sys.argv:
        if a.startswith("--side="):
            ext.debug_set_fast_side_levels(int(a.split("=")[1]))
    cap = ext.max_keypoints(H, W)
    kps = torch.empty(2 * B * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(2 * B * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def run():
        ext.extract_batch_device(2 * B, d_img.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(),
                                 cap, cnt.data_ptr(), stream=s.cuda_stream)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    if "--per-kernel" in sys.argv:
        L.ktimer_reset()
        L.ktimer_select(True)
    t0 = time.perf_counter()
    for _ in range(calls):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"extract: {1e6 * dt / calls:.1f} us per 64-image call, {cnt.float().mean().item():.1f} kp/image")
    if "--per-kernel" in sys.argv:
        L.ktimer_select(False)
        for k, (ms, n) in sorted(L.ktimer_read().items()):
            if n:
                print(f"  {k:14s} {1e3 * ms / calls:9.1f} us/call  {n // calls} launches/call")


if __name__ == "__main__":
    main()
