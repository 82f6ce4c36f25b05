"""The CPU oracle against the committed golden fixtures (regression pin of the checker), and --
marked gpu -- the HIP path against the same fixtures without going through the oracle."""
import numpy as np
import pytest

from golden_io import EXTRACT_CASES, extract_params, load, match_inputs
from oracle import orbref


@pytest.mark.parametrize("case", EXTRACT_CASES)
def test_oracle_extraction_matches_golden(case):
    z = load(case)
    params = extract_params(z)
    ref = orbref.RefExtractor(*params)
    k, d = ref(z["image"])
    assert np.array_equal(k, z["keypoints"])
    assert np.array_equal(d if d is not None else np.zeros((0, 32), np.uint8), z["descriptors"])
    for l in range(params[2]):
        assert np.array_equal(ref.candidates(l), z[f"cand{l}"])
        assert np.array_equal(ref.level_keys(l), z[f"keys{l}"])


def test_oracle_matchers_match_golden():
    z = load("match_320x240.npz")
    F1, F2, mps, last = match_inputs(z)
    ex, ey = (float(v) for v in z["epipole"])
    nm, m12 = orbref.search_for_triangulation(F1, F2, z["F12"], ex, ey, False, True)
    assert nm == int(z["sft_n"]) and np.array_equal(m12, z["sft_m12"])
    nl, bl = orbref.search_by_projection_local(F2, mps, 3.0, 0.8)
    assert nl == int(z["sbp_n"]) and np.array_equal(bl, z["sbp_best"])
    nf, bf = orbref.search_by_projection_lastframe(F2, last, 7.0, False, True)
    assert nf == int(z["sbl_n"]) and np.array_equal(bf, z["sbl_best"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", EXTRACT_CASES)
def test_gpu_extraction_matches_golden(require_gpu, case):
    from orb_slam2_2021_amd import ORBextractor
    z = load(case)
    ext = ORBextractor(*extract_params(z))
    k, d = ext(z["image"])
    for f in ("x", "y", "size", "response", "octave", "class_id"):
        assert np.array_equal(k[f], z["keypoints"][f]), f
    assert np.max(np.abs(k["angle"] - z["keypoints"]["angle"]), initial=0.0) <= 1e-5
    assert np.array_equal(d if d is not None else np.zeros((0, 32), np.uint8), z["descriptors"])


@pytest.mark.gpu
def test_gpu_matchers_match_golden(require_gpu):
    from orb_slam2_2021_amd import ORBmatcher
    z = load("match_320x240.npz")
    F1, F2, mps, last = match_inputs(z)
    ex, ey = (float(v) for v in z["epipole"])
    nm, _, m12 = ORBmatcher(0.6, True).SearchForTriangulation(F1, F2, z["F12"], False, epipole_xy=(ex, ey))
    assert nm == int(z["sft_n"]) and np.array_equal(m12, z["sft_m12"])
    nl, bl = ORBmatcher(0.8).SearchByProjection(F2, mps, 3.0)
    assert nl == int(z["sbp_n"]) and np.array_equal(bl, z["sbp_best"])
    nf, bf = ORBmatcher(0.9, True).SearchByProjection(F2, last, 7.0, bMono=False)
    assert nf == int(z["sbl_n"]) and np.array_equal(bf, z["sbl_best"])
