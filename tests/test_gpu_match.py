"""GPU parity of the ORBmatcher searches (liborbfe.so) against the CPU oracle: match indices and
counts must be identical (integer work: bit-exact bar)."""
import numpy as np
import pytest

from orb_slam2_2021_amd import ORBextractor, ORBmatcher, synth_frame, synth_sequence_frame
from orb_slam2_2021_amd import synthetic as S
from oracle import orbref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kitti_pair():
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    left, right = synth_frame(3, 376, 1241, right=True)
    k1, d1 = ext(left)
    k2, d2 = ext(right)
    return k1, d1, k2, d2, ext.GetScaleFactors(), ext.GetScaleSigmaSquares()


@pytest.fixture(scope="module")
def tum_frame():
    ext = ORBextractor(1000, 1.2, 8, 12, 7)
    k, d = ext(synth_frame(11, 480, 640))
    return k, d, ext.GetScaleFactors(), ext.GetScaleSigmaSquares()


def test_descriptor_distance(require_gpu):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (5000, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (5000, 32), dtype=np.uint8)
    b[:10] = a[:10]
    got = ORBmatcher().DescriptorDistanceBatch(a, b)
    want = np.array([orbref.descriptor_distance(a[i], b[i]) for i in range(len(a))])
    assert np.array_equal(got, want)
    assert got[:10].sum() == 0


@pytest.mark.parametrize("only_stereo", [False, True])
@pytest.mark.parametrize("check_ori", [False, True])
@pytest.mark.parametrize("stereo_frac,epi", [(0.5, None), (0.0, (620.0, 180.0)), (0.3, (150.0, 300.0))])
def test_search_for_triangulation(require_gpu, kitti_pair, only_stereo, check_ori, stereo_frac, epi):
    k1, d1, k2, d2, scale, sigma2 = kitti_pair
    rng = np.random.default_rng(7)
    voc = S.Vocabulary.synthetic()
    cam = S.KITTI_CAM
    t1, t2 = S.pose(), S.pose(tx=-0.537, tz=0.05)
    F1 = S.make_frame(k1, d1, scale, sigma2, 376, 1241, cam, rng, stereo_frac=stereo_frac, tcw=t1)
    F2 = S.make_frame(k2, d2, scale, sigma2, 376, 1241, cam, rng, stereo_frac=stereo_frac, tcw=t2)
    F1.feat_vec = voc.feature_vector(d1, 0)
    F2.feat_vec = voc.feature_vector(d2, 0)
    F12 = S.compute_f12(t1, t2, S.intrinsics(cam))
    ex, ey = epi if epi is not None else (-1.0e7, 185.0)
    m = ORBmatcher(0.6, check_ori)
    nm, pairs, m12 = m.SearchForTriangulation(F1, F2, F12, only_stereo, epipole_xy=(ex, ey))
    nr, r12 = orbref.search_for_triangulation(F1, F2, F12, ex, ey, only_stereo, check_ori)
    assert nm == nr
    assert np.array_equal(m12, r12)
    if not (only_stereo and stereo_frac == 0.0):
        assert nm > 0
    else:
        assert nm == 0  # bOnlyStereo with no stereo keypoint: nothing can match


@pytest.mark.parametrize("k,levels", [(3, 1), (16, 1), (12, 1), (10, 2)])
@pytest.mark.parametrize("same_frame", [False, True])
def test_search_for_triangulation_node_sizes(require_gpu, kitti_pair, k, levels, same_frame):
    """Vocabulary shapes that put ~700, ~125, ~170 and ~20 features in a node: the large-node
    sequential path, the 128-feature boundary of the fixpoint path, and the fixpoint rounds under
    heavy claim conflicts (KF2 = KF1 with shuffled features, so every feature has a twin)."""
    k1, d1, k2, d2, scale, sigma2 = kitti_pair
    if same_frame:
        perm = np.random.default_rng(3).permutation(len(k1))
        k2, d2 = k1[perm], d1[perm]
    rng = np.random.default_rng(11)
    voc = S.Vocabulary.synthetic(k=k, levels=levels)
    t1, t2 = S.pose(), S.pose(tx=-0.537, tz=0.05)
    F1 = S.make_frame(k1, d1, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.4, tcw=t1)
    F2 = S.make_frame(k2, d2, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.4, tcw=t2)
    F1.feat_vec, F2.feat_vec = voc.feature_vector(d1, 0), voc.feature_vector(d2, 0)
    F12 = S.compute_f12(t1, t2, S.intrinsics(S.KITTI_CAM))
    ex, ey = -1.0e7, 185.0
    nm, _, m12 = ORBmatcher(0.6, True).SearchForTriangulation(F1, F2, F12, False, epipole_xy=(ex, ey))
    nr, r12 = orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, True)
    assert nm == nr and np.array_equal(m12, r12)
    assert nm > 0


@pytest.mark.parametrize("big_at", [(3, 259, 262, 300, 511), (0, 1, 2, 257, 258, 259, 260), (300, 301)])
def test_search_for_triangulation_big_nodes_across_chunks(require_gpu, kitti_pair, big_at):
    """FeatureVectors of 520 nodes whose 65-256-feature nodes sit at the given node positions, in and
    past the first 256-node chunk the big-node workgroups scan at a time, so that the workgroups'
    shares of a chunk start at odd and even ranks; KF2 = KF1 shuffled (every feature has a twin)."""
    from orb_slam2_2021_amd.frames import FeatureVector
    k1, d1, _, _, scale, sigma2 = kitti_pair
    n = len(k1)
    rng = np.random.default_rng(23)
    perm = rng.permutation(n)
    k2, d2 = k1[perm], d1[perm]
    node = np.empty(n, np.int64)
    sizes = [70 + 40 * (j % 4) for j in range(len(big_at))]  # 70, 110, 150, 190
    pos = 0
    for j, b in enumerate(big_at):
        node[pos:pos + sizes[j]] = b
        pos += sizes[j]
    small = np.array([b for b in range(520) if b not in big_at])
    node[pos:] = small[np.arange(n - pos) % len(small)]  # every id present: CSR position = node id
    rng.shuffle(node)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    t1, t2 = S.pose(), S.pose(tx=-0.537, tz=0.05)
    F1 = S.make_frame(k1, d1, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.4, tcw=t1)
    F2 = S.make_frame(k2, d2, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.4, tcw=t2)
    F1.feat_vec = FeatureVector.from_assignment(node)
    F2.feat_vec = FeatureVector.from_assignment(node[perm])  # feature q of KF2 is KF1's perm[q]
    F12 = S.compute_f12(t1, t2, S.intrinsics(S.KITTI_CAM))
    ex, ey = -1.0e7, 185.0
    nm, _, m12 = ORBmatcher(0.6, False).SearchForTriangulation(F1, F2, F12, False, epipole_xy=(ex, ey))
    nr, r12 = orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, False)
    assert nm == nr and np.array_equal(m12, r12)
    assert nm > 0


def test_search_for_triangulation_unlisted_features(require_gpu, kitti_pair):
    """Features a FeatureVector does not list -- DBoW2 leaves out stopped words (weight 0,
    TemplatedVocabulary.h:1198-1201) -- are never matched: match12 = -1 for them even when the
    matcher's buffers hold an earlier call's matches."""
    from orb_slam2_2021_amd.frames import FeatureVector
    k1, d1, k2, d2, scale, sigma2 = kitti_pair
    rng = np.random.default_rng(9)
    voc = S.Vocabulary.synthetic()
    t1, t2 = S.pose(), S.pose(tx=-0.537, tz=0.05)
    F1 = S.make_frame(k1, d1, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.5, tcw=t1)
    F2 = S.make_frame(k2, d2, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.5, tcw=t2)
    F12 = S.compute_f12(t1, t2, S.intrinsics(S.KITTI_CAM))
    ex, ey = -1.0e7, 185.0
    m = ORBmatcher(0.6, False)
    full1, full2 = voc.feature_vector(d1, 0), voc.feature_vector(d2, 0)
    F1.feat_vec, F2.feat_vec = full1, full2
    nm0, _, _ = m.SearchForTriangulation(F1, F2, F12, False, epipole_xy=(ex, ey))
    assert nm0 > 0

    def drop(fv, every):  # the same nodes without every `every`-th feature
        d = {}
        for a in range(len(fv.node_ids)):
            kept = [int(i) for i in fv.indices[fv.offsets[a]:fv.offsets[a + 1]] if i % every != 0]
            if kept:
                d[int(fv.node_ids[a])] = kept
        return FeatureVector.from_dict(d)

    for every in (3, 7):
        F1.feat_vec, F2.feat_vec = drop(full1, every), drop(full2, every + 2)
        assert int(F1.feat_vec.offsets[-1]) < len(k1)
        nm, _, m12 = m.SearchForTriangulation(F1, F2, F12, False, epipole_xy=(ex, ey))
        nr, r12 = orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, False)
        assert nm == nr and np.array_equal(m12, r12)
        assert np.all(m12[np.arange(len(k1)) % every == 0] == -1)
        assert nm > 0


def test_search_for_triangulation_epipole_from_poses(require_gpu, kitti_pair):
    k1, d1, k2, d2, scale, sigma2 = kitti_pair
    rng = np.random.default_rng(8)
    voc = S.Vocabulary.synthetic()
    t1, t2 = S.pose(), S.pose(tx=-0.3, tz=1.0, yaw=0.02)
    F1 = S.make_frame(k1, d1, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.0, tcw=t1)
    F2 = S.make_frame(k2, d2, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, stereo_frac=0.0, tcw=t2)
    F1.feat_vec, F2.feat_vec = voc.feature_vector(d1, 0), voc.feature_vector(d2, 0)
    F12 = S.compute_f12(t1, t2, S.intrinsics(S.KITTI_CAM))
    from orb_slam2_2021_amd.frames import epipole
    ex, ey = epipole(F1, F2)
    nm, _, m12 = ORBmatcher(0.6, False).SearchForTriangulation(F1, F2, F12, False)
    nr, r12 = orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, False)
    assert nm == nr and np.array_equal(m12, r12)


@pytest.mark.parametrize("th,seed", [(3.0, 1), (1.0, 2), (5.0, 3)])
def test_search_by_projection_local(require_gpu, tum_frame, th, seed):
    k, d, scale, sigma2 = tum_frame
    rng = np.random.default_rng(seed)
    F = S.make_frame(k, d, scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng, mp_frac=0.1)
    mps = S.make_local_mappoints(F, 20000, rng)
    m = ORBmatcher(0.8)
    nm, best = m.SearchByProjection(F, mps, th)
    nr, rb = orbref.search_by_projection_local(F, mps, th, 0.8)
    rounds, serial = m.last_stats()
    assert nm == nr
    assert np.array_equal(best, rb)
    assert nm > 100
    assert serial == 0, f"fixpoint did not settle in {rounds} rounds"


def test_search_by_projection_local_serial_fallback(require_gpu, tum_frame):
    k, d, scale, sigma2 = tum_frame
    rng = np.random.default_rng(5)
    F = S.make_frame(k, d, scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng, mp_frac=0.1)
    mps = S.make_local_mappoints(F, 3000, rng, match_frac=0.6)
    m = ORBmatcher(0.8)
    m.set_max_rounds(1)
    nm, best = m.SearchByProjection(F, mps, 3.0)
    nr, rb = orbref.search_by_projection_local(F, mps, 3.0, 0.8)
    assert m.last_stats()[1] == 1
    assert nm == nr and np.array_equal(best, rb)


@pytest.mark.parametrize("mono", [False, True])
@pytest.mark.parametrize("check_ori", [False, True])
@pytest.mark.parametrize("motion", [(0.01, 0.0, 0.02, 0.01), (0.0, 0.0, 0.3, 0.0), (0.0, 0.0, -0.3, 0.0)])
def test_search_by_projection_lastframe(require_gpu, tum_frame, mono, check_ori, motion):
    k, d, scale, sigma2 = tum_frame
    rng = np.random.default_rng(11)
    C = S.make_frame(k, d, scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng, mp_frac=0.05,
                     tcw=S.pose(tx=motion[0], ty=motion[1], tz=motion[2], yaw=motion[3]))
    last = S.make_lastframe(C, 1500, rng, None)
    m = ORBmatcher(0.9, check_ori)
    nm, best = m.SearchByProjection(C, last, 7.0, bMono=mono)
    nr, rb = orbref.search_by_projection_lastframe(C, last, 7.0, mono, check_ori)
    assert nm == nr
    assert np.array_equal(best, rb)
    assert nm > 50


@pytest.fixture(scope="module")
def kitti_seq_frame():
    """The left image of frame 5 of the bench's driving sequence (1241x376), KITTI extractor settings."""
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = ext(synth_sequence_frame(0x0C3, 5, 376, 1241))
    return k, d, ext.GetScaleFactors(), ext.GetScaleSigmaSquares()


# Tracking::TrackWithMotionModel's thresholds (Tracking.cc:900-904): 7 for stereo, 15 otherwise; the
# camera moving forward (tz = -1 m: LastFrame ahead of mb, the search from nLastOctave up), backward
# (from level 0 to nLastOctave) and nearly still (nLastOctave - 1 .. + 1); ORBmatcher.cc:1366-1410
@pytest.mark.parametrize("mono,th", [(False, 7.0), (True, 15.0)])
@pytest.mark.parametrize("check_ori", [False, True])
@pytest.mark.parametrize("tz", [-1.0, 1.0, 0.05])
def test_search_by_projection_lastframe_kitti(require_gpu, kitti_seq_frame, mono, th, check_ori, tz):
    k, d, scale, sigma2 = kitti_seq_frame
    rng = np.random.default_rng(int(100 * tz) + 107)
    C = S.make_frame(k, d, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, mp_frac=0.0,
                     tcw=S.pose(tz=tz, yaw=0.01))
    last = S.make_lastframe(C, 1800, rng, None)
    m = ORBmatcher(0.9, check_ori)  # Tracking.cc:889
    nm, best = m.SearchByProjection(C, last, th, bMono=mono)
    nr, rb = orbref.search_by_projection_lastframe(C, last, th, mono, check_ori)
    assert nm == nr and np.array_equal(best, rb)
    assert nm > 100


@pytest.mark.parametrize("sweep", [(0, 0, 0), (16, 0, 0), (64, 0, 5), (32, 1, 0)])
@pytest.mark.parametrize("check_ori", [False, True])
def test_search_by_projection_lastframe_sweep_knobs(require_gpu, kitti_seq_frame, check_ori, sweep):
    """The last-frame search (first-minimum mode, TH_HIGH, rotation filter) through k_sbp_sweep with
    its test knobs -- small chunks, a 5-entry cache (queries past it walk the grid), the per-chunk
    sequential walk: the oracle's result, with the rotation filter's undo codes."""
    from orb_slam2_2021_amd import _lib as L
    k, d, scale, sigma2 = kitti_seq_frame
    rng = np.random.default_rng(211)
    C = S.make_frame(k, d, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, mp_frac=0.0,
                     tcw=S.pose(tz=-1.0, yaw=0.01))
    last = S.make_lastframe(C, 1800, rng, None)
    m = ORBmatcher(0.9, check_ori)
    L.check(L.lib().orbfe_debug_matcher_set_sweep(m._h, *sweep), "set_sweep")
    nm, best = m.SearchByProjection(C, last, 15.0, bMono=True)
    nr, rb = orbref.search_by_projection_lastframe(C, last, 15.0, True, check_ori)
    assert nm == nr and np.array_equal(best, rb)
    assert nm > 100


@pytest.mark.parametrize("n_last,retried", [(30, True), (1800, False)])
@pytest.mark.parametrize("mono,th", [(False, 7.0), (True, 15.0)])
def test_motion_model_retry(require_gpu, kitti_seq_frame, n_last, retried, mono, th):
    """Tracking.cc:905-911: below 20 matches the search runs again at 2 th on a cleared frame."""
    k, d, scale, sigma2 = kitti_seq_frame
    rng = np.random.default_rng(n_last)
    C = S.make_frame(k, d, scale, sigma2, 376, 1241, S.KITTI_CAM, rng, mp_frac=0.2, tcw=S.pose(tz=-1.0))
    last = S.make_lastframe(C, n_last, rng, None, match_frac=0.5)
    m = ORBmatcher(0.9, True)
    nm, best, th_used = m.SearchByProjectionMotionModel(C, last, th, mono)
    nr, rb, th_ref = orbref.motion_model_search(C, last, th, mono, True)
    assert (th_used, nm) == (th_ref, nr) and np.array_equal(best, rb)
    assert (th_used == 2 * th) == retried
    assert (C.mp_state == 0).all()  # the fill before each pass (Tracking.cc:897, 909)


def test_empty_inputs(require_gpu, tum_frame):
    k, d, scale, sigma2 = tum_frame
    rng = np.random.default_rng(0)
    F = S.make_frame(k[:0], d[:0], scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng)
    mps = S.make_local_mappoints(S.make_frame(k, d, scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng), 100, rng)
    nm, best = ORBmatcher(0.8).SearchByProjection(F, mps, 3.0)
    assert nm == 0 and (best == -1).all()
    F2 = S.make_frame(k, d, scale, sigma2, 480, 640, S.ARDUCAM_CAM, rng)
    empty = S.make_local_mappoints(F2, 0, rng)
    nm, best = ORBmatcher(0.8).SearchByProjection(F2, empty, 3.0)
    assert nm == 0 and len(best) == 0
