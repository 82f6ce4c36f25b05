"""k_octree phase clocks of a SMALL call (the C2 / tracking path: 512-thread blocks, latency
schedule) on a profiling build (-DORBFE_OCT_PROF=1, ORBFE_LIB pointing at it): N images (default 1)
of the bench's C2 image (frame 0 of its driving sequence; OCT_IMG=synth for synth_frame(3)),
device-resident, per level the mean/max of each phase in microseconds.
usage: ORBFE_LIB=... python profiles/scripts/oct_prof_small.py [reps] [N]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from orb_slam2_2021_amd import ORBextractor, synth_frame  # noqa: E402
from orb_slam2_2021_amd import _lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n, H, W = (int(sys.argv[2]) if len(sys.argv) > 2 else 1), 376, 1241
    dev = torch.device("cuda", 0)
    if os.environ.get("OCT_IMG") == "synth":
        im = synth_frame(3, H, W)
    else:
        from orb_slam2_2021_amd.extractor import synth_sequence_frame
        im = synth_sequence_frame(0x0C3, 0, H, W)
        im = im[0] if isinstance(im, tuple) else im
    imgs = torch.from_numpy(np.stack([im] * n)).to(dev)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    if os.environ.get("OCT_THREADS"):
        ext.debug_set_octree_threads(int(os.environ["OCT_THREADS"]), 256)
    if os.environ.get("ORBFE_OCT_SPLIT"):  # the octree launch split (orbfe_debug_set_octree_split)
        ext.debug_set_octree_split(int(os.environ["ORBFE_OCT_SPLIT"]))
    cap = ext.max_keypoints(H, W)
    kps = torch.empty(n * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(n * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    lib = L.lib()
    fn = lib.orbfe_debug_octree_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(64 * 16 * 16, np.uint64)
    names = ["scan", "gather", "initial", "passes", "refine", "retain"]
    acc = []
    for r in range(reps + 1):
        ext.extract_batch_device(n, imgs.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(), cap,
                                 cnt.data_ptr())
        torch.cuda.synchronize()
        L.check(fn(buf.ctypes.data, buf.size), "octree_prof")
        if r:
            acc.append(buf.reshape(64, 16, 16).astype(np.int64).copy())
    a = np.stack(acc)  # reps x img x level x 16
    t = a.astype(np.float64) / 100.0  # us
    start = t[..., 0]
    print(f"launch span (first block start .. last block end): "
          f"{np.mean([(t[i, :, :8, 6].max() - start[i, :, :8].min()) for i in range(len(acc))]):.1f} us")
    print("level  n_keys passes rounds  S   " + "  ".join(f"{x:>13s}" for x in names) + "   total(mean/max)")
    for l in range(8):
        c = a[..., l, 7]
        nk, passes, rounds, S = c & 0xffffff, (c >> 24) & 0xff, (c >> 32) & 0xffff, (c >> 48) & 0xffff
        ph = [t[..., l, k + 1] - t[..., l, k] for k in range(6)]
        tot = t[..., l, 6] - t[..., l, 0]
        print(f"{l:5d} {nk.mean():7.0f} {passes.mean():6.1f} {rounds.mean():6.1f} {S.mean():5.0f}  " +
              "  ".join(f"{p.mean():6.1f}/{p.max():6.1f}" for p in ph) + f"   {tot.mean():6.1f}/{tot.max():6.1f}")
    sub = ["flag scan", "sort", "child counts", "stop scan", "partition", "build"]
    print("first refinement round (us):  " + "  ".join(f"{x:>12s}" for x in sub) +
          "     first pass: splits   scan   rest")
    for l in range(8):
        r = [t[..., l, 8] - t[..., l, 4]] + [t[..., l, k + 1] - t[..., l, k] for k in range(8, 13)]
        p1 = [t[..., l, 14] - t[..., l, 3], t[..., l, 15] - t[..., l, 14]]
        print(f"{l:5d}                         " + "  ".join(f"{x.mean():12.1f}" for x in r) +
              f"     {p1[0].mean():12.1f} {p1[1].mean():6.1f}")
    if os.environ.get("ORBFE_OCT_PROF_PASS"):  # a build with -DORBFE_OCT_PROF_PASS=k: marks 14/15
        k = os.environ["ORBFE_OCT_PROF_PASS"]  # bracket full pass k (zero when a level has fewer)
        d = t[..., :8, 15] - t[..., :8, 14]
        print(f"full pass {k} (us, mean/max per level): " +
              "  ".join(f"{d[..., l].mean():5.1f}/{d[..., l].max():5.1f}" for l in range(8)))
        cyc, sn = a[..., :8, 12].astype(np.float64), a[..., :8, 13]
        ns, nk = (sn & 0xffff).astype(np.float64), (sn >> 16).astype(np.float64)
        print("  wave 0's wave splits (shader clocks per split / keys per split / splits, per level): " +
              "  ".join(f"{(cyc[..., l] / np.maximum(ns[..., l], 1)).mean():6.0f}/"
                        f"{(nk[..., l] / np.maximum(ns[..., l], 1)).mean():4.0f}/{ns[..., l].mean():3.1f}"
                        for l in range(8)))
        print("  sub-steps (us, thread 0's wavefront): thread-split  wave-split  barrier  scan  build")
        for l in range(8):
            m = [14, 8, 9, 10, 11, 15]
            print(f"  {l:5d}  " + "  ".join(f"{(t[..., l, m[i + 1]] - t[..., l, m[i]]).mean():10.1f}"
                                         for i in range(5)))


if __name__ == "__main__":
    main()
