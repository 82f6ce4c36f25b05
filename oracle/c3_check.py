"""Oracle check of one C3 sub-batch (TEST INFRASTRUCTURE ONLY: used by tests/test_gpu_c3.py and
bench.py's parity leg as the checker, never by the product).

Runs the reference chain on the CPU from the same input images and KeyFrame state --
ORBextractor::operator() (orbref.cpp), TemplatedVocabulary::transform (orbref_vocab.cpp),
[Frame::ComputeStereoMatches,] ORBmatcher::SearchForTriangulation (orbref.cpp) -- and compares
every stage of the GPU's outputs (orb_slam2_2021_amd.pipeline.C3Pipeline.to_host): keypoint
x/y/size/response/octave/class_id exact and angle within 1e-5, descriptors, BowVector ids and
weights (bit-equal doubles), FeatureVector CSR, mvuRight (bit-equal) and match12 exact.
"""
from __future__ import annotations

import time

import numpy as np

from oracle import orbref


def check_c3(images, gpu, ref_voc, u_right, mp_state, scale, sigma2, cam, F12, epipole, levelsup=4,
             nfeatures=2000, ini_th=20, min_th=7, stereo=False, mb=0.0, pairs="stereo"):
    """images: (2B, H, W) uint8, lefts then rights; u_right / mp_state: (2B, cap) KeyFrame state
    as the pipeline read it; pairs: "stereo" (ComputeBoW on all 2B images, SearchForTriangulation
    on (left_i, right_i)) or "kf" (ComputeBoW on the B lefts, SearchForTriangulation on
    (left_t, left_t+1)), as orb_slam2_2021_amd.pipeline.C3Pipeline runs them. Returns per-stage
    flags, the first mismatch, and the CPU seconds."""
    from orb_slam2_2021_amd.frames import FeatureVector, Frame
    t0 = time.perf_counter()
    n_img, H, W = images.shape
    B = n_img // 2
    n_vocab = B if pairs == "kf" else n_img
    pair_idx = [(i, i + 1) for i in range(B - 1)] if pairs == "kf" else [(i, B + i) for i in range(B)]
    ex_l = orbref.RefExtractor(nfeatures, 1.2, 8, ini_th, min_th)
    ex_r = orbref.RefExtractor(nfeatures, 1.2, 8, ini_th, min_th)
    flags = {"keypoints": True, "descriptors": True, "bow": True, "feature_vector": True,
             "match12": True}
    if stereo:
        flags["u_right"] = True
    first = None

    def fail(stage, where):
        nonlocal first
        flags[stage] = False
        if first is None:
            first = f"{stage} differs at {where}"

    tab = ex_l.tables()
    frames = [None] * n_img
    max_angle = 0.0
    for p in range(B):
        for ex, i in ((ex_l, p), (ex_r, B + p)):
            k, d = ex(images[i])
            d = d if d is not None else np.zeros((0, 32), np.uint8)
            gk, gd = gpu["keypoints"][i], gpu["descriptors"][i]
            if len(gk) != len(k) or any(not np.array_equal(gk[f], k[f]) for f in
                                        ("x", "y", "size", "response", "octave", "class_id")) \
                    or (len(k) and np.max(np.abs(gk["angle"] - k["angle"])) > 1e-5):
                fail("keypoints", f"image {i}")
            if len(gk) == len(k) and len(k):
                max_angle = max(max_angle, float(np.max(np.abs(gk["angle"].astype(np.float64) - k["angle"]))))
            if not np.array_equal(gd, d):
                fail("descriptors", f"image {i}")
            n = len(k)
            F = Frame(keys_un=k, descriptors=d, u_right=u_right[i, :n], mp_state=mp_state[i, :n],
                      scale_factors=scale, level_sigma2=sigma2, min_x=0.0, max_x=float(W), min_y=0.0,
                      max_y=float(H), **cam)
            if i < n_vocab:
                words, weights, fv = ref_voc.transform(d, levelsup)
                gw, gt = gpu["bow"][i]
                if not (np.array_equal(gw, words) and np.array_equal(gt.view(np.uint64), weights.view(np.uint64))):
                    fail("bow", f"image {i}")
                gi, go, gx = gpu["fv"][i]
                if not (np.array_equal(gi, fv[0]) and np.array_equal(go, fv[1]) and np.array_equal(gx, fv[2])):
                    fail("feature_vector", f"image {i}")
                F.feat_vec = FeatureVector(*fv)
            frames[i] = F
        if stereo:  # Frame.cc:125 on the two extractors' pyramids: mvuRight of the left KeyFrame
            F1, F2 = frames[p], frames[B + p]
            lv = [ex_l.level(i) for i in range(8)]
            rv = [ex_r.level(i) for i in range(8)]
            ur, _ = orbref.compute_stereo_matches(F1.keys_un, F1.descriptors, F2.keys_un, F2.descriptors,
                                                  lv, rv, tab["scale"], tab["inv_scale"], mb, cam["bf"])
            if not np.array_equal(ur.view(np.uint32), gpu["u_right"][p].view(np.uint32)):
                fail("u_right", f"pair {p}")
            F1.u_right = ur
    for q, (a, b) in enumerate(pair_idx):
        nm, m12 = orbref.search_for_triangulation(frames[a], frames[b], F12, epipole[0], epipole[1], False, False)
        if nm != int(gpu["nmatches"][q]) or not np.array_equal(m12, gpu["match12"][q]):
            fail("match12", f"pair {q} (images {a}, {b})")
    out = dict(flags)
    out["all"] = all(flags.values())
    # the north star allows 1e-5 on the angle; 0.0 here means every angle is bit-identical too
    out["max_angle_abs_diff"] = max_angle
    out["first_mismatch"] = first
    out["images"] = n_img
    out["pairs"] = len(pair_idx)
    out["pairing"] = pairs
    out["cpu_seconds"] = round(time.perf_counter() - t0, 2)
    return out
