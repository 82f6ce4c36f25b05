"""The C3 matching chain alone (KeyFrame::ComputeBoW of the 32 left KeyFrames + SearchForTriangulation
of the 31 KeyFrame pairs, the bench default), repeated on one extracted sub-batch, for rocprofv3
kernel traces / PMC passes of the vocabulary and SFT kernels without the extraction beside them:
python profiles/scripts/match_only.py [reps] [--stereo-pairs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from orb_slam2_2021_amd import ORBextractor, synth_frame, synth_sequence_frame
from orb_slam2_2021_amd import synthetic as S
from orb_slam2_2021_amd.pipeline import build_c3
from orb_slam2_2021_amd.vocabulary import ORBVocabulary


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 50
    pairs = "stereo" if "--stereo-pairs" in sys.argv else "kf"
    B, H, W = 32, 376, 1241
    host = np.zeros((2 * B, H, W), np.uint8)
    for i in range(B):
        if pairs == "kf":
            host[i], host[B + i] = synth_sequence_frame(0x0C3, i, H, W, right=True)
        else:
            host[i], host[B + i] = synth_frame(i, H, W, right=True)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    tree = S.Vocabulary.synthetic_orbvoc()
    voc = ORBVocabulary.from_tree(tree)
    pipe, _ = build_c3(ext, tree, voc, B, H, W, 0, stereo=True, pairs=pairs)
    d = torch.from_numpy(host).cuda()
    torch.cuda.set_stream(pipe.stream)
    pipe.run(d.data_ptr())
    torch.cuda.synchronize()
    o = pipe.last
    m = pipe.mstream
    for _ in range(3):
        pipe._match(o, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        pipe._match(o, None)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    nm = o.nm.cpu().numpy()[:pipe.n_pairs]
    print(f"matching chain ({pairs}): {1e6 * dt:.1f} us per sub-batch, {pipe.n_pairs} pairs, "
          f"{nm.mean():.1f} matches per pair")
    # SearchForTriangulation alone (k_sft_nodes + k_sft_finish), HIP events per call
    import ctypes
    from orb_slam2_2021_amd import _lib as L
    lib = L.lib()
    ts = []
    for r in range(reps + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(m)
        L.check(lib.orbfe_search_for_triangulation_batch_device(
            o.matcher._h, pipe.n_pairs, ctypes.cast(o.pairs, ctypes.c_void_p), 0, ctypes.c_void_p(m.cuda_stream)),
            "sft batch")
        b.record(m)
        if r >= 3:
            ts.append((a, b))
    torch.cuda.synchronize()
    us = [1e3 * a.elapsed_time(b) for a, b in ts]
    print(f"SearchForTriangulation x{pipe.n_pairs}: {np.median(us):.1f} us per call (median of {reps}), "
          f"min {min(us):.1f}")


if __name__ == "__main__":
    main()
