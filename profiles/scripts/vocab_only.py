"""KeyFrame::ComputeBoW of the C3 sub-batch's 32 left KeyFrames alone (k_vocab_descend + k_vocab),
repeated on one extracted sub-batch; HIP events per call. For phase-cost builds of k_vocab
(-DORBFE_VOCAB_DIAG, wrong outputs that nothing reads here): python vocab_only.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from orb_slam2_2021_amd import ORBextractor, synth_sequence_frame
from orb_slam2_2021_amd import synthetic as S
from orb_slam2_2021_amd.pipeline import build_c3
from orb_slam2_2021_amd.vocabulary import ORBVocabulary


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    B, H, W = 32, 376, 1241
    host = np.zeros((2 * B, H, W), np.uint8)
    for i in range(B):
        host[i], host[B + i] = synth_sequence_frame(0x0C3, i, H, W, right=True)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    tree = S.Vocabulary.synthetic_orbvoc()
    voc = ORBVocabulary.from_tree(tree)
    pipe, _ = build_c3(ext, tree, voc, B, H, W, 0, stereo=True, pairs="kf")
    d = torch.from_numpy(host).cuda()
    torch.cuda.set_stream(pipe.stream)
    pipe.run(d.data_ptr())
    torch.cuda.synchronize()
    o, m = pipe.last, pipe.mstream
    ts = []
    for r in range(reps + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(m)
        pipe._vocab(o, m)
        b.record(m)
        if r >= 3:
            ts.append((a, b))
    torch.cuda.synchronize()
    us = [1e3 * a.elapsed_time(b) for a, b in ts]
    print(f"ComputeBoW x{pipe.n_vocab}: {np.median(us):.1f} us per call (median of {reps}), min {min(us):.1f}")


if __name__ == "__main__":
    main()
