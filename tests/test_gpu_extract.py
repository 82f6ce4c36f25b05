"""GPU parity of ORBextractor::operator() (liborbfe.so HIP kernels) against the CPU oracle.

Bar (north star): bit-exact 32-byte descriptors; keypoint set, order, coordinates, octave, size and
response exact; angle within 1e-5 (exact in practice: fastAtan2 runs the same float op sequence).
Every stage is checked so a mismatch names its kernel: pyramid level bytes (k_resize), FAST
candidates in octree input order (k_fast), octree survivors (k_octree), final keypoints and
descriptors (k_describe).
"""
import numpy as np
import pytest

from orb_slam2_2021_amd import ORBextractor, synth_frame, ORBFE_RESIZE_SCALAR
from orb_slam2_2021_amd._lib import KEYPOINT_DTYPE
from oracle import orbref
from oracle.orbref import RefExtractor

pytestmark = pytest.mark.gpu

ANGLE_TOL = 1e-5


def assert_same_extraction(ext, ref, img, image_index=0, got=None):
    kg, dg = got if got is not None else ext(img)
    kr, dr = ref(img)
    for l in range(ref.nlevels):
        lr = ref.level(l)
        lg = ext.level(l, image=image_index)
        assert lg.shape == lr.shape, f"level {l} shape"
        bad = np.argwhere(lg != lr)
        assert len(bad) == 0, f"k_resize: level {l} differs at {len(bad)} px, first {bad[:5].tolist()}"
    for l in range(ref.nlevels):
        br = orbref.gaussian_blur7(ref.level(l))
        bg = ext.debug_blurred(l, image=image_index)
        bad = np.argwhere(bg != br)
        assert len(bad) == 0, f"k_blur: level {l} differs at {len(bad)} px, first {bad[:5].tolist()}"
    for l in range(ref.nlevels):
        cr, cg = ref.candidates(l), ext.debug_candidates(l, image=image_index)
        assert len(cg) == len(cr), f"k_fast: level {l} candidate count {len(cg)} vs {len(cr)}"
        assert np.array_equal(cg, cr), f"k_fast: level {l} first diff at {np.argmax(cg != cr)}"
    for l in range(ref.nlevels):
        sr, sg = ref.level_keys(l), ext.debug_level_keys(l, image=image_index)
        assert len(sg) == len(sr), f"k_octree: level {l} survivor count {len(sg)} vs {len(sr)}"
        assert np.array_equal(sg, sr), f"k_octree: level {l} first diff at {np.argmax(sg != sr)}"
    assert len(kg) == len(kr)
    for f in ("x", "y", "size", "response", "octave", "class_id"):
        assert np.array_equal(kg[f], kr[f]), f"keypoint field {f}"
    assert np.max(np.abs(kg["angle"] - kr["angle"]), initial=0.0) <= ANGLE_TOL
    if len(kr):
        nbad = int(np.sum(np.any(dg != dr, axis=1)))
        assert nbad == 0, f"k_describe: {nbad} of {len(kr)} descriptors differ"
    return len(kr)


@pytest.mark.parametrize("index", [0, 1, 7])
def test_kitti_shape_bit_exact(require_gpu, index):
    img = synth_frame(index, 376, 1241)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    ref = RefExtractor(2000, 1.2, 8, 20, 7)
    n = assert_same_extraction(ext, ref, img)
    assert n >= 2000


def test_right_image_and_tum_shape(require_gpu):
    _, right = synth_frame(5, 376, 1241, right=True)
    assert_same_extraction(ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7), right)
    img = synth_frame(11, 480, 640)
    assert_same_extraction(ORBextractor(1000, 1.2, 8, 12, 7), RefExtractor(1000, 1.2, 8, 12, 7), img)


def test_other_parameters(require_gpu):
    img = synth_frame(21, 400, 700)
    for params in [(500, 1.2, 4, 20, 7), (3000, 1.3, 6, 15, 5), (2000, 1.2, 8, 7, 20)]:
        assert_same_extraction(ORBextractor(*params), RefExtractor(*params), img)


def test_scalar_resize_mode(require_gpu):
    img = synth_frame(2, 376, 1241)
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.set_resize_mode(ORBFE_RESIZE_SCALAR)
    ref.set_resize_mode(ORBFE_RESIZE_SCALAR)
    assert_same_extraction(ext, ref, img)


@pytest.mark.parametrize("shape", [(376, 1241), (480, 640), (260, 1500), (900, 700)])
def test_pyramid_shapes(require_gpu, shape):
    """k_copy0 + the per-level k_resize_win launches give the reference pyramid on wide, tall and
    KITTI/TUM shapes."""
    img = synth_frame(9, *shape)
    assert_same_extraction(ORBextractor(1000, 1.2, 8, 20, 7), RefExtractor(1000, 1.2, 8, 20, 7), img)


@pytest.mark.parametrize("params,shape", [((800, 1.1, 12, 20, 7), (480, 640)), ((300, 1.2, 1, 20, 7), (240, 333)),
                                          ((500, 1.2, 2, 20, 7), (377, 643)), ((1500, 1.5, 5, 20, 7), (601, 1023))])
def test_pyramid_level_counts(require_gpu, params, shape):
    """1, 2, 5 and 12 levels on odd widths (scale factors 1.1-1.5); every level's bytes, and the rest
    of the extraction, vs the oracle."""
    img = synth_frame(17, *shape)
    assert_same_extraction(ORBextractor(*params), RefExtractor(*params), img)


def test_flat_and_sparse_images(require_gpu):
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    flat = np.full((376, 1241), 128, np.uint8)
    kg, dg = ext(flat)
    assert len(kg) == 0 and dg is None
    assert_same_extraction(ext, ref, flat)
    sparse = np.full((376, 1241), 90, np.uint8)
    sparse[100:140, 300:330] = 200
    sparse[250:262, 900:1000] = 10
    assert_same_extraction(ext, ref, sparse)
    noise = np.random.default_rng(3).integers(0, 256, (376, 1241), dtype=np.uint8)
    assert_same_extraction(ext, ref, noise)


@pytest.mark.parametrize("cap", [0, 1024])
def test_octree_global_key_path(require_gpu, cap):
    """DistributeOctTree keeps a level's keys in LDS up to a capacity and in global scratch beyond
    it; force the global path for every level (0) or for the large levels only (1024)."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_octree_key_cap(cap)
    assert_same_extraction(ext, ref, synth_frame(3, 376, 1241))
    noise = np.random.default_rng(5).integers(0, 256, (376, 1241), dtype=np.uint8)
    assert_same_extraction(ext, ref, noise)


@pytest.mark.parametrize("split,lds,threads", [(0, None, 256), (1, None, 256), (3, None, 256), (4, None, 256),
                                               (7, None, 256), (8, None, 256), (4, (64, 32), 256),
                                               (4, (48, 24), 256), (4, None, 512), (0, None, 1024),
                                               (4, (48, 24), 512)])
def test_octree_launch_split(require_gpu, split, lds, threads):
    """DistributeOctTree as one launch (0, 8) or two (levels 0..k-1 at the 80 KiB LDS plan, k.. at
    the 40 KiB one) over an 8-image batch: the same survivors, on textured and noise images (noise
    pushes the small levels' key counts past the half plan's LDS capacity, onto the global path)."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_octree_split(split)
    ext.debug_set_octree_threads(512, threads)  # the batch's block size
    if lds:  # smaller plans: more keys through the global path
        ext.debug_set_octree_lds(*lds)
    # (the split applies to device-resident batches of 8+ images: one such batch, every image checked)
    import torch
    noise = np.random.default_rng(9).integers(0, 256, (376, 1241), dtype=np.uint8)
    imgs = np.stack([synth_frame(4 + i, 376, 1241) for i in range(7)] + [noise])
    n, H, W = imgs.shape
    cap = ext.max_keypoints(H, W)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(imgs).to(dev)
    kps = torch.empty(n * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(n * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ext.extract_batch_device(n, d_in.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(), cap,
                             cnt.data_ptr())
    torch.cuda.synchronize()
    C = cnt.cpu().numpy()
    K = kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(n, cap)
    D = desc.cpu().numpy().reshape(n, cap, 32)
    for i in reversed(range(n)):
        got = (K[i, :C[i]], D[i, :C[i]] if C[i] else None)
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=got)


@pytest.mark.parametrize("blur_mode,k,n", [(0, 1, 1), (1, 1, 1), (0, 2, 1), (1, 2, 2), (0, 3, 2), (0, 7, 4),
                                            (0, 0, 1)])
def test_latency_schedule(require_gpu, blur_mode, k, n):
    """The latency schedule (FAST and DistributeOctTree of levels 0..k-1 on the side stream beside the
    main stream's levels k..; calls of fewer than 8 images; k = 0 the throughput schedule): every
    stage equals the oracle, for both blur placements, several k and 1-4 images, on textured and
    noise images."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_latency_schedule(k)
    ext.debug_set_blur_mode(blur_mode)
    noise = np.random.default_rng(11).integers(0, 256, (376, 1241), dtype=np.uint8)
    imgs = [synth_frame(21 + i, 376, 1241) for i in range(n - 1)] + [noise]
    for _ in range(2):  # the second round through the same handle (its streams and events reused)
        outs = ext.extract_batch(imgs) if n > 1 else [ext(imgs[0])]
    for i in reversed(range(n)):
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


@pytest.mark.parametrize("threads,cap", [(256, -1), (512, -1), (1024, -1), (1024, 0), (1024, 1024), (512, 0)])
def test_octree_block_sizes(require_gpu, threads, cap):
    """DistributeOctTree's block of a call of fewer than 8 images: 512 threads (the default), 1024,
    or the batches' 256 -- the same survivors on KITTI-, TUM- and odd-shaped images, textured and
    noise, one image and three per call, with the keys in LDS or forced to the global path (cap 0:
    every level, 1024: the large ones)."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_octree_threads(threads, 256)
    if cap >= 0:
        ext.debug_set_octree_key_cap(cap)
    rng = np.random.default_rng(17)
    for shape in ((376, 1241), (480, 640), (301, 517)):
        imgs = [synth_frame(31, *shape), rng.integers(0, 256, shape, dtype=np.uint8), synth_frame(32, *shape)]
        assert_same_extraction(ext, ref, imgs[0])
        outs = ext.extract_batch(imgs)
        for i in reversed(range(len(imgs))):
            assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


@pytest.mark.parametrize("small,batch,cap", [(64, 48, -1), (128, 16, -1), (1, 128, -1), (64, 64, 0)])
def test_octree_serial_threshold(require_gpu, small, batch, cap):
    """DistributeOctTree with other thread-serial / wavefront split thresholds
    (orbfe_debug_set_octree_serial) for small calls and batches: the same survivors, one image,
    three per call and an 8-image device batch, keys in LDS or (cap 0) on the global path."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_octree_serial(small, batch)
    if cap >= 0:
        ext.debug_set_octree_key_cap(cap)
    rng = np.random.default_rng(23)
    for shape in ((376, 1241), (301, 517)):
        imgs = [synth_frame(41, *shape), rng.integers(0, 256, shape, dtype=np.uint8), synth_frame(42, *shape)]
        assert_same_extraction(ext, ref, imgs[0])
        outs = ext.extract_batch(imgs)
        for i in reversed(range(len(imgs))):
            assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])
    imgs = [synth_frame(80 + i, 376, 1241) for i in range(8)]
    outs = _extract_device_batch(ext, imgs)
    for i in (0, 5, 7):
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


def _extract_device_batch(ext, imgs):
    import torch
    imgs = np.stack(imgs)
    n, H, W = imgs.shape
    cap = ext.max_keypoints(H, W)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(imgs).to(dev)
    kps = torch.empty(n * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(n * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ext.extract_batch_device(n, d_in.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(), cap,
                             cnt.data_ptr())
    torch.cuda.synchronize()
    C = cnt.cpu().numpy()
    K = kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(n, cap)
    D = desc.cpu().numpy().reshape(n, cap, 32)
    return [(K[i, :C[i]], D[i, :C[i]] if C[i] else None) for i in range(n)]


@pytest.mark.parametrize("tiles", [(2, 2), (4, 4), (8, 6), (16, 8), (3, 5), (32, 24), (1, 1)])
def test_pyramid_tiles(require_gpu, tiles):
    """ComputePyramid's levels 1.. in one k_pyramid launch (each workgroup builds its tile of every
    level with the previous level in LDS and the halo recomputed): the same bytes as the per-level
    chain on KITTI, TUM and odd shapes, 1 image (the small calls' plan) and an 8-image device batch
    (the batches' plan), textured and noise; (1, 1) needs more LDS than a tile may hold and falls
    back to the chain."""
    rng = np.random.default_rng(23)
    for params, shape in (((2000, 1.2, 8, 20, 7), (376, 1241)), ((1000, 1.2, 8, 20, 7), (480, 640)),
                          ((500, 1.2, 8, 20, 7), (301, 517)), ((800, 1.1, 12, 20, 7), (480, 640)),
                          ((1000, 2.0, 3, 20, 7), (600, 1241)), ((500, 1.2, 2, 20, 7), (377, 643))):
        ext, ref = ORBextractor(*params), RefExtractor(*params)
        ext.debug_set_pyramid_tiles(tiles, tiles)
        img = synth_frame(33, *shape)
        assert_same_extraction(ext, ref, img)
        imgs = [synth_frame(34 + i, *shape) for i in range(7)] + [rng.integers(0, 256, shape, dtype=np.uint8)]
        outs = _extract_device_batch(ext, imgs)
        for i in reversed(range(len(imgs))):
            assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


@pytest.mark.parametrize("fast_side", [2, 4])
def test_fast_side_merge(require_gpu, fast_side):
    """Batches with the side stream's FAST levels 1..k-1 in one launch (orbfe_debug_set_fast_side_merge)
    instead of one per level: the same candidates and keypoints, 8-image device batch."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_fast_side_levels(fast_side)
    ext.debug_set_fast_side_merge(True)
    rng = np.random.default_rng(29)
    imgs = [synth_frame(70 + i, 376, 1241) for i in range(7)] + [rng.integers(0, 256, (376, 1241), dtype=np.uint8)]
    outs = _extract_device_batch(ext, imgs)
    for i in reversed(range(len(imgs))):
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


@pytest.mark.parametrize("params", [(1000, 2.0, 3, 20, 7), (1000, 2.5, 3, 20, 7)])
def test_large_scale_factors(require_gpu, params):
    """Scale 2.0 still fits the 8-byte window resize (k_resize_win); 2.5 takes the byte-gather
    k_resize path."""
    img = synth_frame(13, 600, 1241)
    assert_same_extraction(ORBextractor(*params), RefExtractor(*params), img)


@pytest.mark.parametrize("zc_in,zc_out", [(True, True), (True, False), (False, True), (False, False)])
def test_host_calls_alternating_images(require_gpu, zc_in, zc_out):
    """Single-image host-buffer calls through one handle with the image changing every call (A B C A B
    C ...): k_copy0 reading the staging buffer over PCIe (zero copy in, the default) or after an H2D
    copy must see each call's bytes, and the results written straight into the pinned host mirror
    (zero copy out, the default) or copied down must be each call's own -- every call equals the
    oracle."""
    ext, ref = ORBextractor(1000, 1.2, 8, 20, 7), RefExtractor(1000, 1.2, 8, 20, 7)
    ext.debug_set_zero_copy(zc_in, zc_out)
    imgs = [synth_frame(50 + i, 240, 333) for i in range(3)]
    expect = [ref(im) for im in imgs]
    for r in range(4):
        for i, im in enumerate(imgs):
            kg, dg = ext(im)
            kr, dr = expect[i]
            assert len(kg) == len(kr), f"round {r} image {i}: {len(kg)} vs {len(kr)} keypoints"
            for f in ("x", "y", "octave", "response"):
                assert np.array_equal(kg[f], kr[f]), f"round {r} image {i}: field {f}"
            assert np.array_equal(dg, dr), f"round {r} image {i}: descriptors"
    assert_same_extraction(ext, ref, imgs[-1], got=(kg, dg))


def test_schedule_autotune_decides_and_stays_exact(require_gpu):
    """Calls of fewer than 8 images time the two-stream latency schedule against the launch stream
    alone over their first host-buffer calls (per image count) and keep one: the choice is made by
    the 16th call, every call of both arms equals the oracle, and switching the autotune off
    resets it (two streams)."""
    ext, ref = ORBextractor(1000, 1.2, 8, 20, 7), RefExtractor(1000, 1.2, 8, 20, 7)
    imgs = [synth_frame(60 + i, 240, 333) for i in range(2)]
    expect = [ref(im) for im in imgs]
    assert ext.debug_schedule_choice(1) == -1
    for i in range(18):
        kg, dg = ext(imgs[i % 2])
        kr, dr = expect[i % 2]
        assert len(kg) == len(kr) and np.array_equal(kg["x"], kr["x"]) and np.array_equal(dg, dr), f"call {i}"
    assert ext.debug_schedule_choice(1) in (0, 1)
    assert ext.debug_schedule_choice(2) == -1  # per image count
    outs = ext.extract_batch(imgs)
    for i in range(2):
        assert np.array_equal(outs[i][1], expect[i][1])
    ext.debug_set_schedule_autotune(False)
    assert ext.debug_schedule_choice(1) == -1
    kg, dg = ext(imgs[0])
    assert np.array_equal(dg, expect[0][1])


def test_empty_image(require_gpu):
    k, d = ORBextractor(2000, 1.2, 8, 20, 7)(np.zeros((0, 0), np.uint8))
    assert len(k) == 0 and d is None


def test_batch_equals_single(require_gpu):
    imgs = [synth_frame(i, 376, 1241) for i in range(4)]
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    ref = RefExtractor(2000, 1.2, 8, 20, 7)
    outs = ext.extract_batch(imgs)
    for i in reversed(range(4)):  # the debug hooks read the batch just run
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


def test_host_batch_pipeline(require_gpu):
    """orbfe_extract_batch with >= 8 host images takes the chunked staging / H2D / pieced D2H path:
    every image equals its own single-image extraction, with a caller pitch wider than the rows,
    and every image's pyramid stays readable afterwards (each chunk extracted into its own slots)."""
    import ctypes
    from orb_slam2_2021_amd import _lib as L
    n, rows, cols, step = 19, 240, 333, 352
    imgs = [synth_frame(40 + i, rows, cols) for i in range(n)]
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.max_keypoints(rows, cols)
    buf = np.zeros((n, rows, step), np.uint8)
    for i in range(n):
        buf[i, :, :cols] = imgs[i]
        buf[i, :, cols:] = 255 - i  # padding bytes the extraction must never read
    kps = np.empty(n * cap, L.KEYPOINT_DTYPE)
    desc = np.empty((n * cap, 32), np.uint8)
    counts = np.zeros(n, np.int32)
    arr = (ctypes.c_void_p * n)(*[buf[i].ctypes.data for i in range(n)])
    L.check(L.lib().orbfe_extract_batch(ext._h, n, ctypes.cast(arr, ctypes.c_void_p), rows, cols,
                                        ctypes.c_size_t(step), L.ptr(kps), L.ptr(desc), cap, L.ptr(counts)),
            "orbfe_extract_batch")
    levels = [[ext.level(l, image=i).copy() for l in range(8)] for i in range(n)]
    single = ORBextractor(1000, 1.2, 8, 20, 7)
    for i in range(n):
        k1, d1 = single(imgs[i])
        c = int(counts[i])
        assert c == len(k1), i
        kb, db = kps[i * cap:i * cap + c], desc[i * cap:i * cap + c]
        for f in ("x", "y", "size", "response", "octave", "angle"):
            assert np.array_equal(kb[f], k1[f]), (i, f)
        assert np.array_equal(db, d1), i
        for l in range(8):
            assert np.array_equal(levels[i][l], single.level(l)), (i, l)
    # one image through the oracle as well
    kr, dr = RefExtractor(1000, 1.2, 8, 20, 7)(imgs[7])
    c = int(counts[7])
    assert c == len(kr) and np.array_equal(desc[7 * cap:7 * cap + c], dr)


@pytest.mark.parametrize("k", [1, 2, 0])
def test_small_device_batch_latency_schedule(require_gpu, k):
    """orbfe_extract_batch_device with fewer than 8 images takes the latency schedule too (k side
    levels; 0 = the throughput schedule): every image equals the oracle."""
    import torch
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_latency_schedule(k)
    imgs = np.stack([synth_frame(90 + i, 376, 1241) for i in range(3)])
    n, H, W = imgs.shape
    cap = ext.max_keypoints(H, W)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(imgs).to(dev)
    kps = torch.empty(n * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(n * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ext.extract_batch_device(n, d_in.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(), cap,
                             cnt.data_ptr())
    torch.cuda.synchronize()
    C = cnt.cpu().numpy()
    K = kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(n, cap)
    D = desc.cpu().numpy().reshape(n, cap, 32)
    for i in reversed(range(n)):
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=(K[i, :C[i]], D[i, :C[i]] if C[i] else None))


def test_small_calls_after_large_on_one_handle(require_gpu):
    """A small host call's results come down in one copy of the output block's prefix only while the
    block is not much larger than the call; after a 9-image call on the same handle, single images
    and pairs take the separate copies, and a later larger call regrows the block: every result
    equals a fresh handle's (and one image the oracle's)."""
    rows, cols = 240, 333
    ext, fresh = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
    seq = [1, 9, 1, 2, 1, 12, 1]
    for j, n in enumerate(seq):
        imgs = [synth_frame(70 + 13 * j + i, rows, cols) for i in range(n)]
        outs = ext.extract_batch(imgs) if n > 1 else [ext(imgs[0])]
        for i in range(n):
            k1, d1 = fresh(imgs[i])
            kb, db = outs[i]
            assert len(kb) == len(k1), (j, i)
            for f in ("x", "y", "size", "response", "octave", "angle"):
                assert np.array_equal(kb[f], k1[f]), (j, i, f)
            assert np.array_equal(db, d1), (j, i)
    kr, dr = RefExtractor(1000, 1.2, 8, 20, 7)(imgs[0])
    assert np.array_equal(outs[0][1], dr)


@pytest.mark.parametrize("prefetch", [False, True])
@pytest.mark.parametrize("n", [1, 3, 9])
def test_mvimagepyramid_views_held_at_once(require_gpu, prefetch, n):
    """orbfe_get_level's contract (include/orbfe.h): every level of every image of the last call
    stays valid together until the next extract call, as the reference's mvImagePyramid[0..7]
    (ORBextractor.h:100) does for Frame::ComputeStereoMatches (Frame.cc:529,620-640), which reads
    levels of any octave of both extractors in one pass. All n x 8 views are taken first (no copy)
    and only then compared with the oracle's levels; the lazy path (one DMA per image on its first
    access) and the prefetch path (orbfe_extractor_set_host_pyramid, copies beside the extraction);
    1 image (orbfe_extract's path), 3 (one launch group), 9 (the chunked copy-stream pipeline).
    After the next call the views show the new call's pyramids."""
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    ext.set_host_pyramid(prefetch)
    ref = RefExtractor(2000, 1.2, 8, 20, 7)
    for rnd in range(2):
        imgs = [synth_frame(70 + 10 * rnd + i, 376, 1241) for i in range(n)]
        if n == 1:
            ext(imgs[0])
        else:
            ext.extract_batch(imgs)
        views = [[ext.level_view(l, image=i) for l in range(8)] for i in range(n)]
        spans = sorted((v.__array_interface__["data"][0], v.__array_interface__["data"][0] +
                        (v.shape[0] - 1) * v.strides[0] + v.shape[1]) for row in views for v in row)
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "two levels share host memory"
        for i in reversed(range(n)):
            ref(imgs[i])
            for l in range(8):
                assert np.array_equal(views[i][l], ref.level(l)), (rnd, i, l)


def test_repeatable(require_gpu):
    img = synth_frame(9, 376, 1241)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    a = ext(img)
    b = ext(img)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_candidate_total_matches_per_level_lists(require_gpu):
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    imgs = [synth_frame(i, 376, 1241) for i in range(3)]
    ext.extract_batch(imgs)
    want = sum(len(ext.debug_candidates(l, image=i)) for i in range(3) for l in range(8))
    assert ext.debug_candidate_total() == want > 0


def test_library_umax_equals_oracle(require_gpu):
    """liborbfe's IC_Angle circle table = the oracle's (pinned to ORBextractor.cc:457-472 by
    tests/test_reference_pins.py)."""
    from orb_slam2_2021_amd import _lib as L
    from oracle.orbref import RefExtractor
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    u = np.zeros(16, np.int32)
    L.check(L.lib().orbfe_debug_get_umax(ext._h, L.ptr(u)), "get_umax")
    assert u.tolist() == RefExtractor(2000, 1.2, 8, 20, 7).tables()["umax"].tolist()


def test_blur_after_octree(require_gpu):
    """GaussianBlur after DistributeOctTree on the launch stream (the several-handle placement): the
    same blurred levels, keypoints and descriptors as the oracle."""
    ext, ref = ORBextractor(2000, 1.2, 8, 20, 7), RefExtractor(2000, 1.2, 8, 20, 7)
    ext.debug_set_blur_mode(1)
    assert_same_extraction(ext, ref, synth_frame(4, 376, 1241))
    imgs = [synth_frame(30 + i, 376, 1241) for i in range(3)]
    outs = ext.extract_batch(imgs)
    for i in reversed(range(3)):
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=outs[i])


def test_device_input_odd_pitch_and_alignment(require_gpu):
    """extract_batch_device on images at an odd byte offset with an odd row pitch (k_copy0's
    unaligned loads and last-dword byte path) equals the oracle, image by image."""
    import torch
    from orb_slam2_2021_amd import _lib as L
    n, rows, cols, pitch = 3, 376, 1241, 1247
    imgs = [synth_frame(60 + i, rows, cols) for i in range(n)]
    buf = np.full(n * rows * pitch + 8, 77, np.uint8)
    for i in range(n):
        v = buf[1 + i * rows * pitch:1 + (i + 1) * rows * pitch].reshape(rows, pitch)
        v[:, :cols] = imgs[i]
    d = torch.from_numpy(buf).to("cuda")
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ext.max_keypoints(rows, cols)
    kps = torch.empty(n * cap * 28, dtype=torch.uint8, device="cuda")
    desc = torch.empty(n * cap * 32, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    ext.extract_batch_device(n, d.data_ptr() + 1, rows * pitch, rows, cols, pitch, kps.data_ptr(),
                             desc.data_ptr(), cap, cnt.data_ptr())
    torch.cuda.synchronize()
    K = kps.cpu().numpy().view(L.KEYPOINT_DTYPE).reshape(n, cap)
    D = desc.cpu().numpy().reshape(n, cap, 32)
    C = cnt.cpu().numpy()
    ref = RefExtractor(2000, 1.2, 8, 20, 7)
    for i in reversed(range(n)):
        c = int(C[i])
        assert_same_extraction(ext, ref, imgs[i], image_index=i, got=(K[i, :c], D[i, :c]))


def test_launch_graph_replay(require_gpu):
    """The launch sequence replayed from hipGraphs (orbfe_extractor_set_graphs(1)) equals direct
    launches (the default): host path
    (orbfe_extract, captured once then replayed), device batches into alternating output sets on a
    caller's stream (one graph per argument set), a new output pointer (a new capture), the kernel
    timer on (direct launches inside a graphed handle), and graphs off."""
    import torch
    from orb_slam2_2021_amd import _lib as L
    imgs = [synth_frame(60 + i, 376, 1241) for i in range(3)]
    a, b = ORBextractor(2000, 1.2, 8, 20, 7), ORBextractor(2000, 1.2, 8, 20, 7)
    a.set_graphs(True)
    for img in imgs + imgs:
        ka, da = a(img)
        kb, db = b(img)
        for f in ("x", "y", "size", "response", "octave", "angle"):
            assert np.array_equal(ka[f], kb[f]), f
        assert np.array_equal(da, db)
    cap_, hits, held = a.debug_graph_stats()
    assert cap_ == 1 and hits == 5 and held == 1, (cap_, hits, held)
    assert b.debug_graph_stats() == (0, 0, 0)
    # device batches: 2 images per call, two output sets, a caller stream
    dev = torch.device("cuda", 0)
    n, H, W = 2, 376, 1241
    cap = a.max_keypoints(H, W)
    d_in = torch.from_numpy(np.stack(imgs[:n])).to(dev)
    outs = [(torch.empty(n * cap * 28, dtype=torch.uint8, device=dev), torch.empty(n * cap * 32, dtype=torch.uint8, device=dev),
             torch.zeros(n, dtype=torch.int32, device=dev)) for _ in range(3)]
    s = torch.cuda.Stream(dev)

    def run(e, o):
        e.extract_batch_device(n, d_in.data_ptr(), H * W, H, W, W, o[0].data_ptr(), o[1].data_ptr(), cap,
                               o[2].data_ptr(), stream=s.cuda_stream)

    for k in range(6):
        run(a, outs[k % 2])
    run(b, outs[2])
    torch.cuda.synchronize()
    for o in outs[:2]:
        assert torch.equal(o[2], outs[2][2])
        for i in range(n):
            c = int(outs[2][2][i])
            assert torch.equal(o[0][i * cap * 28:(i * cap + c) * 28], outs[2][0][i * cap * 28:(i * cap + c) * 28])
            assert torch.equal(o[1][i * cap * 32:(i * cap + c) * 32], outs[2][1][i * cap * 32:(i * cap + c) * 32])
    cap2, hits2, held2 = a.debug_graph_stats()
    # (the 2-image batch reallocated the handle's scratch, which drops the 1-image host-path graph)
    assert cap2 == 3 and hits2 == 5 + 4 and held2 == 2, (cap2, hits2, held2)
    # the kernel timer on: launches go direct (no capture, no replay)
    L.ktimer_select(True)
    try:
        run(a, outs[0])
        torch.cuda.synchronize()
    finally:
        L.ktimer_select(False)
        L.ktimer_read()
    assert a.debug_graph_stats() == (cap2, hits2, held2)
    assert torch.equal(outs[0][2], outs[2][2])
    # graphs off drops them
    a.set_graphs(False)
    assert a.debug_graph_stats()[2] == 0
