"""ORBextractor on MI355X -- host mirror of include/ORBextractor.h over liborbfe.so.

Same constructor arguments, getters and call semantics as the reference class
(include/ORBextractor.h:56-100, src/ORBextractor.cc:413-473, 1041-1103): calling the extractor on
an 8-bit grayscale image returns its keypoints (cv::KeyPoint fields, level order) and the N x 32
descriptor matrix. All work runs in the HIP kernels of liborbfe.so.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_size_t, c_void_p
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

KeyPoints = np.ndarray  # structured, dtype KEYPOINT_DTYPE


class ORBextractor:
    HARRIS_SCORE = 0  # ORBextractor.h:51-54 (enum kept for API parity)
    FAST_SCORE = 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, device: int = 0):
        self._lib = L.lib()
        h = c_void_p()
        L.check(self._lib.orbfe_extractor_create(int(nfeatures), float(scaleFactor), int(nlevels),
                                                 int(iniThFAST), int(minThFAST), int(device),
                                                 byref(h)), "orbfe_extractor_create")
        self._h = h
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        self.device = int(device)
        n = self.nlevels
        self._scale = np.zeros(n, np.float32)
        self._inv = np.zeros(n, np.float32)
        self._s2 = np.zeros(n, np.float32)
        self._is2 = np.zeros(n, np.float32)
        self._fpl = np.zeros(n, np.int32)
        L.check(self._lib.orbfe_get_scale_tables(self._h, L.ptr(self._scale), L.ptr(self._inv),
                                                 L.ptr(self._s2), L.ptr(self._is2),
                                                 L.ptr(self._fpl)), "orbfe_get_scale_tables")
        self._last_shape: Optional[Tuple[int, int]] = None

    # ---- lifetime -------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.orbfe_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- getters (ORBextractor.h:70-98) ---------------------------------------------------
    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return self.scaleFactor

    def GetScaleFactors(self) -> np.ndarray:
        return self._scale.copy()

    def GetInverseScaleFactors(self) -> np.ndarray:
        return self._inv.copy()

    def GetScaleSigmaSquares(self) -> np.ndarray:
        return self._s2.copy()

    def GetInverseScaleSigmaSquares(self) -> np.ndarray:
        return self._is2.copy()

    @property
    def mnFeaturesPerLevel(self) -> np.ndarray:
        return self._fpl.copy()

    def set_resize_mode(self, mode: int) -> None:
        L.check(self._lib.orbfe_extractor_set_resize_mode(self._h, int(mode)), "set_resize_mode")

    def max_keypoints(self, rows: int, cols: int) -> int:
        return L.check(self._lib.orbfe_max_keypoints(self._h, int(rows), int(cols)),
                       "orbfe_max_keypoints")

    # ---- operator() -----------------------------------------------------------------------
    def __call__(self, image: np.ndarray, mask=None) -> Tuple[KeyPoints, Optional[np.ndarray]]:
        """operator()(image, mask, keypoints, descriptors). The mask is ignored, as in the
        reference (ORBextractor.h:65). Returns (keypoints, descriptors); descriptors is None when
        no keypoint was found (the reference releases the Mat, ORBextractor.cc:1062-1063)."""
        img = np.asarray(image)
        if img.size == 0:
            return np.zeros(0, L.KEYPOINT_DTYPE), None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects a CV_8UC1 image")  # assert at :1048
        img = np.ascontiguousarray(img)
        rows, cols = img.shape
        cap = self.max_keypoints(rows, cols)
        kps = np.zeros(cap, L.KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = c_int()
        L.check(self._lib.orbfe_extract(self._h, L.ptr(img), rows, cols, c_size_t(img.strides[0]),
                                        L.ptr(kps), cap, L.ptr(desc), byref(n)), "orbfe_extract")
        self._last_shape = (rows, cols)
        k = n.value
        return kps[:k].copy(), (desc[:k].copy() if k else None)

    def extract_batch(self, images: Sequence[np.ndarray]) -> List[Tuple[KeyPoints, np.ndarray]]:
        """Independent operator() calls on same-shaped images in one launch sequence."""
        imgs = [np.ascontiguousarray(np.asarray(i, np.uint8)) for i in images]
        if not imgs:
            return []
        rows, cols = imgs[0].shape
        if any(i.shape != (rows, cols) for i in imgs):
            raise ValueError("extract_batch needs same-shaped images")
        cap = self.max_keypoints(rows, cols)
        B = len(imgs)
        kps = np.empty(B * cap, L.KEYPOINT_DTYPE)
        desc = np.empty((B * cap, 32), np.uint8)
        counts = np.zeros(B, np.int32)
        arr = (c_void_p * B)(*[i.ctypes.data for i in imgs])
        L.check(self._lib.orbfe_extract_batch(self._h, B, ctypes.cast(arr, c_void_p), rows, cols,
                                              c_size_t(cols), L.ptr(kps), L.ptr(desc), cap,
                                              L.ptr(counts)), "orbfe_extract_batch")
        self._last_shape = (rows, cols)
        out = []
        for b in range(B):
            k = int(counts[b])
            out.append((kps[b * cap:b * cap + k].copy(), desc[b * cap:b * cap + k].copy()))
        return out

    def extract_batch_device(self, n_images: int, d_imgs: int, image_stride: int, rows: int,
                             cols: int, pitch: int, d_kps: int, d_desc: int, cap: int,
                             d_counts: int, stream: Optional[int] = None) -> None:
        """Device-resident batch (all int arguments are device addresses); async on `stream`."""
        L.check(self._lib.orbfe_extract_batch_device(
            self._h, int(n_images), c_void_p(d_imgs), c_size_t(image_stride), int(rows), int(cols),
            c_size_t(pitch), c_void_p(d_kps), c_void_p(d_desc), int(cap), c_void_p(d_counts),
            c_void_p(stream or 0)), "orbfe_extract_batch_device")
        self._last_shape = (rows, cols)

    # ---- Frame::ComputeStereoMatches (src/Frame.cc:522-700) -------------------------------
    def compute_stereo_matches(self, kps_l: KeyPoints, desc_l: np.ndarray, kps_r: KeyPoints,
                               desc_r: np.ndarray, mbf: float, mb: float, right: "ORBextractor" = None,
                               image_left: int = 0, image_right: Optional[int] = None
                               ) -> Tuple[np.ndarray, np.ndarray]:
        """Frame::ComputeStereoMatches (Frame.cc:522-700): (mvuRight, mvDepth) of the left keypoints.
        The left pyramid is image `image_left` of this extractor's last call; the right pyramid is
        image `image_right` of `right`'s last call (default: this extractor, image 1 -- e.g. after
        extract_batch([left, right]); with a separate right extractor, its image 0).
        mb: the reference uses the Frame's mb before assigning it (Frame.cc:125 vs :149); pass
        mbf / fx, or 0 for an unbounded disparity range."""
        other = self if right is None else right
        if image_right is None:
            image_right = 1 if other is self else 0
        kl = np.ascontiguousarray(kps_l, L.KEYPOINT_DTYPE)
        kr = np.ascontiguousarray(kps_r, L.KEYPOINT_DTYPE)
        dl = np.ascontiguousarray(desc_l if desc_l is not None else np.zeros((0, 32)), np.uint8)
        dr = np.ascontiguousarray(desc_r if desc_r is not None else np.zeros((0, 32)), np.uint8)
        n = len(kl)
        ur = np.full(n, -1.0, np.float32)
        dep = np.full(n, -1.0, np.float32)
        L.check(self._lib.orbfe_compute_stereo_matches(
            self._h, int(image_left), other._h, int(image_right), L.ptr(kl), L.ptr(dl), n,
            L.ptr(kr), L.ptr(dr), len(kr), float(mbf), float(mb), L.ptr(ur), L.ptr(dep)),
            "orbfe_compute_stereo_matches")
        return ur, dep

    def stereo_frame(self, left: np.ndarray, right: np.ndarray, mbf: float, mb: float):
        """The stereo Frame constructor's hot path (Frame.cc:113-125): ExtractORB(0, left),
        ExtractORB(1, right), ComputeStereoMatches. Returns (kps_l, desc_l, kps_r, desc_r,
        u_right, depth)."""
        l = np.ascontiguousarray(np.asarray(left, np.uint8))
        r = np.ascontiguousarray(np.asarray(right, np.uint8))
        if l.shape != r.shape or l.ndim != 2:
            raise ValueError("stereo_frame needs two same-shaped CV_8UC1 images")
        rows, cols = l.shape
        if l.size == 0:
            e = np.zeros(0, L.KEYPOINT_DTYPE)
            return e, None, e.copy(), None, np.zeros(0, np.float32), np.zeros(0, np.float32)
        cap = self.max_keypoints(rows, cols)
        kl = np.zeros(cap, L.KEYPOINT_DTYPE)
        kr = np.zeros(cap, L.KEYPOINT_DTYPE)
        dl = np.zeros((cap, 32), np.uint8)
        dr = np.zeros((cap, 32), np.uint8)
        ur = np.zeros(cap, np.float32)
        dep = np.zeros(cap, np.float32)
        nl, nr = c_int(), c_int()
        L.check(self._lib.orbfe_stereo_frame(self._h, L.ptr(l), L.ptr(r), rows, cols, c_size_t(cols),
                                             float(mbf), float(mb), L.ptr(kl), L.ptr(dl), byref(nl),
                                             L.ptr(kr), L.ptr(dr), byref(nr), cap, L.ptr(ur),
                                             L.ptr(dep)), "orbfe_stereo_frame")
        self._last_shape = (rows, cols)
        a, b = nl.value, nr.value
        return (kl[:a].copy(), dl[:a].copy() if a else None, kr[:b].copy(),
                dr[:b].copy() if b else None, ur[:a].copy(), dep[:a].copy())

    def compute_stereo_matches_batch_device(self, n_pairs: int, left0: int, right0: int, d_kps: int,
                                            d_desc: int, d_counts: int, cap: int, mbf: float,
                                            mb: float, d_u_right: int, d_depth: int,
                                            stream: Optional[int] = None) -> None:
        """Device-resident ComputeStereoMatches over pairs (left0 + p, right0 + p) of the last
        extract_batch_device call; outputs at p*cap + i. Async on `stream`."""
        L.check(self._lib.orbfe_compute_stereo_matches_batch_device(
            self._h, int(n_pairs), int(left0), int(right0), c_void_p(d_kps), c_void_p(d_desc),
            c_void_p(d_counts), int(cap), float(mbf), float(mb), c_void_p(d_u_right),
            c_void_p(d_depth), c_void_p(stream or 0)), "orbfe_compute_stereo_matches_batch_device")

    @property
    def stream(self) -> int:
        return self._lib.orbfe_extractor_stream(self._h) or 0

    def wait_pyramid(self, stream: int) -> None:
        """Make `stream` wait for the pyramid of this handle's last extract call
        (orbfe_extractor_pyramid_event): call right after the extract call."""
        L.check(self._lib.orbfe_stream_wait_event(c_void_p(stream or 0),
                                                  c_void_p(self._lib.orbfe_extractor_pyramid_event(self._h))),
                "orbfe_stream_wait_event")

    # ---- mvImagePyramid (ORBextractor.h:100) --------------------------------------------
    def level_view(self, level: int, image: int = 0) -> np.ndarray:
        """mvImagePyramid[level] of image `image` of the last call as a view of the handle's host
        block (no copy): valid until the next extract call, like the reference's cv::Mat headers."""
        p = c_void_p()
        r, c, s = c_int(), c_int(), c_size_t()
        L.check(self._lib.orbfe_get_level(self._h, image, level, byref(p), byref(r), byref(c),
                                          byref(s)), "orbfe_get_level")
        buf = (ctypes.c_uint8 * ((r.value - 1) * s.value + c.value)).from_address(p.value)
        return np.lib.stride_tricks.as_strided(np.frombuffer(buf, np.uint8), (r.value, c.value), (s.value, 1))

    def level(self, level: int, image: int = 0) -> np.ndarray:
        return self.level_view(level, image).copy()

    def set_host_pyramid(self, on: bool = True) -> None:
        """orbfe_extractor_set_host_pyramid: later host-buffer calls copy each pyramid to the host
        beside the extraction, so mvImagePyramid costs no copy of its own."""
        L.check(self._lib.orbfe_extractor_set_host_pyramid(self._h, 1 if on else 0), "set_host_pyramid")

    def set_graphs(self, on: bool) -> None:
        """orbfe_extractor_set_graphs: replay each extract call's launch sequence as a hipGraph
        captured per argument set; off (the default) launches every kernel directly."""
        L.check(self._lib.orbfe_extractor_set_graphs(self._h, 1 if on else 0), "set_graphs")

    def debug_graph_stats(self) -> tuple:
        """(graph captures, graph replays, graphs held) of this handle."""
        import numpy as np
        out = np.zeros(3, np.int64)
        L.check(self._lib.orbfe_debug_graph_stats(self._h, out.ctypes.data), "graph_stats")
        return tuple(int(x) for x in out)

    @property
    def mvImagePyramid(self) -> List[np.ndarray]:
        return [self.level(l) for l in range(self.nlevels)]

    # ---- instrumentation ----------------------------------------------------------------
    def debug_candidates(self, level: int, image: int = 0) -> np.ndarray:
        n = c_int()
        L.check(self._lib.orbfe_debug_get_candidates(self._h, image, level, None, 0, byref(n)),
                "debug_candidates")
        out = np.zeros(max(n.value, 1), np.uint32)
        L.check(self._lib.orbfe_debug_get_candidates(self._h, image, level, L.ptr(out), len(out),
                                                     byref(n)), "debug_candidates")
        return out[:n.value]
    def debug_candidate_total(self) -> int:
        """FAST candidates over every image and level of the last call."""
        t = ctypes.c_longlong()
        L.check(self._lib.orbfe_debug_candidate_total(self._h, byref(t)), "debug_candidate_total")
        return t.value

    def debug_level_keys(self, level: int, image: int = 0) -> np.ndarray:
        n = c_int()
        L.check(self._lib.orbfe_debug_get_level_keys(self._h, image, level, None, 0, byref(n)),
                "debug_level_keys")
        out = np.zeros(max(n.value, 1), np.uint32)
        L.check(self._lib.orbfe_debug_get_level_keys(self._h, image, level, L.ptr(out), len(out),
                                                     byref(n)), "debug_level_keys")
        return out[:n.value]

    def debug_blurred(self, level: int, image: int = 0) -> np.ndarray:
        ref = self.level(level, image)
        out = np.zeros(ref.shape, np.uint8)
        L.check(self._lib.orbfe_debug_get_blurred(self._h, image, level, L.ptr(out), out.size),
                "debug_blurred")
        return out

    def debug_set_octree_key_cap(self, cap: int) -> None:
        """Limit the keys DistributeOctTree keeps in LDS (0: global-memory path; <0: auto)."""
        L.check(self._lib.orbfe_debug_set_octree_key_cap(self._h, int(cap)), "set_octree_key_cap")

    def debug_set_fast_side_levels(self, k: int) -> None:
        """FAST of levels 0..k-1 on the side stream as each level is built (k <= 0: the default, 3)."""
        L.check(self._lib.orbfe_debug_set_fast_side_levels(self._h, int(k)), "set_fast_side_levels")

    def debug_set_octree_split(self, k: int) -> None:
        """DistributeOctTree in two launches for batches of 8+ images, levels 0..k-1 at 80 KiB of LDS
        per block and k.. at 40 KiB (default 5; k <= 0: one launch of every level at 80 KiB)."""
        L.check(self._lib.orbfe_debug_set_octree_split(self._h, int(k)), "set_octree_split")

    def debug_set_octree_threads(self, small_calls: int, batches: int = 256) -> None:
        """DistributeOctTree's block size (256 / 512 / 1024) for calls of fewer than 8 images (512
        default) and for batches of 8+ (256 default)."""
        L.check(self._lib.orbfe_debug_set_octree_threads(self._h, int(small_calls), int(batches)),
                "set_octree_threads")

    def debug_set_octree_serial(self, small_calls: int, batches: int = 48) -> None:
        """DistributeOctTree: nodes of at most this many keys split by one thread, larger ones by a
        wavefront (1..128), for calls of fewer than 8 images / batches of 8+."""
        L.check(self._lib.orbfe_debug_set_octree_serial(self._h, int(small_calls), int(batches)),
                "set_octree_serial")

    def debug_set_fast_side_merge(self, on: bool) -> None:
        """Batches: the side stream's FAST levels 1..k-1 in one launch after level k-1 is built."""
        L.check(self._lib.orbfe_debug_set_fast_side_merge(self._h, int(bool(on))), "set_fast_side_merge")

    def debug_set_schedule_autotune(self, on: bool) -> None:
        """Calls of fewer than 8 images: time the latency schedule on two streams against one stream
        over the first host-buffer calls and keep the faster (default on); off: always two."""
        L.check(self._lib.orbfe_debug_set_schedule_autotune(self._h, int(bool(on))), "set_schedule_autotune")

    def debug_schedule_choice(self, n_images: int = 1) -> int:
        """-1 still timing, 0 two streams, 1 the launch stream alone (calls of n_images images)."""
        return int(self._lib.orbfe_debug_schedule_choice(self._h, int(n_images)))

    def debug_set_zero_copy(self, inp: bool, out: Optional[bool] = None) -> None:
        """Host-buffer calls of fewer than 8 images: k_copy0 reads the staged image from pinned host
        memory, and the kernels write the results into the pinned host mirror (both default) instead
        of H2D / D2H copies (out defaults to inp)."""
        out = inp if out is None else out
        L.check(self._lib.orbfe_debug_set_zero_copy(self._h, int(bool(inp)), int(bool(out))), "set_zero_copy")

    def debug_set_pyramid_tiles(self, small=(0, 0), batch=(0, 0)) -> None:
        """ComputePyramid's levels 1.. in one k_pyramid launch of tx x ty tiles per image for calls of
        fewer than 8 images / batches of 8+ ((0, 0): one resize launch per level)."""
        L.check(self._lib.orbfe_debug_set_pyramid_tiles(self._h, int(small[0]), int(small[1]), int(batch[0]),
                                                        int(batch[1])), "set_pyramid_tiles")

    def debug_set_latency_schedule(self, k: int) -> None:
        """Calls of fewer than 8 images: FAST and DistributeOctTree of levels 0..k-1 on the side stream
        beside the main stream's levels k.. (default 1; k <= 0: the throughput schedule)."""
        L.check(self._lib.orbfe_debug_set_latency_schedule(self._h, int(k)), "set_latency_schedule")

    def debug_set_octree_lds(self, hi_kb: int, lo_kb: int) -> None:
        """LDS budgets (KiB per block) of the octree launches below / from the split (80 / 40)."""
        L.check(self._lib.orbfe_debug_set_octree_lds(self._h, int(hi_kb), int(lo_kb)), "set_octree_lds")

    def debug_set_fast_wpb(self, side_wpb: int, main_wpb: int) -> None:
        """k_fast cells per workgroup: side-stream launches (default 4), the rest (default 1)."""
        L.check(self._lib.orbfe_debug_set_fast_wpb(self._h, int(side_wpb), int(main_wpb)), "set_fast_wpb")

    def debug_set_blur_mode(self, mode: int) -> None:
        """GaussianBlur placement: 0 side stream beside DistributeOctTree (default), 1 launch stream
        after it (several handles sharing one side stream)."""
        L.check(self._lib.orbfe_debug_set_blur_mode(self._h, int(mode)), "set_blur_mode")

    def set_side_stream(self, stream: int) -> None:
        """Run the side-stream work on `stream` (a hipStream_t address; 0 restores the handle's own)."""
        L.check(self._lib.orbfe_set_side_stream(self._h, c_void_p(stream or 0)), "set_side_stream")

    def debug_set_inline_side(self, on: bool = True) -> None:
        """Run the side-stream work (k_blur, early FAST levels) on the launch stream."""
        L.check(self._lib.orbfe_debug_set_inline_side(self._h, 1 if on else 0), "set_inline_side")

    def geometry(self, rows: int, cols: int) -> np.ndarray:
        info = np.zeros(7 * self.nlevels, np.int32)
        L.check(self._lib.orbfe_debug_geometry(self._h, rows, cols, L.ptr(info), len(info)),
                "geometry")
        return info.reshape(self.nlevels, 7)


def register_host(a: np.ndarray) -> None:
    """orbfe_host_register: page-lock a (C-contiguous) numpy buffer the host-buffer entry points
    then DMA from / to directly (images; keypoint and descriptor outputs with cap equal to
    max_keypoints). Keep the array alive and call unregister_host before dropping it."""
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("register_host needs a C-contiguous array")
    L.check(L.lib().orbfe_host_register(c_void_p(a.ctypes.data), c_size_t(a.nbytes)), "orbfe_host_register")


def unregister_host(a: np.ndarray) -> None:
    L.check(L.lib().orbfe_host_unregister(c_void_p(a.ctypes.data)), "orbfe_host_unregister")


def synth_frame(index: int, rows: int = 376, cols: int = 1241, n_rects: int = 0,
                right: bool = False):
    """Seeded synthetic KITTI-shaped frame (orbfe_synth.h). Returns left or (left, right)."""
    lib = L.lib()
    left = np.zeros((rows, cols), np.uint8)
    r = np.zeros((rows, cols), np.uint8) if right else None
    L.check(lib.orbfe_synth_frame(int(index), rows, cols, int(n_rects), L.ptr(left),
                                  L.ptr(r) if right else None, c_size_t(cols)), "orbfe_synth_frame")
    return (left, r) if right else left


def synth_sequence_frame(seq: int, t: int, rows: int = 376, cols: int = 1241, cam: dict = None,
                         step_z: float = 1.0, right: bool = False):
    """Frame t of a seeded driving sequence (orbfe_synth_sequence_frame): the camera moves step_z m
    along +z per frame, so frames t and t+1 are the C3 KeyFrame pair of SURVEY 8(d). `cam` holds
    fx, fy, cx, cy and bf (baseline = bf / fx); KITTI-like by default. Returns left or (left, right)."""
    from .synthetic import KITTI_CAM
    cam = cam or KITTI_CAM
    lib = L.lib()
    left = np.zeros((rows, cols), np.uint8)
    r = np.zeros((rows, cols), np.uint8) if right else None
    L.check(lib.orbfe_synth_sequence_frame(int(seq), int(t), rows, cols, cam["fx"], cam["fy"], cam["cx"], cam["cy"],
                                           cam["bf"] / cam["fx"], float(step_z), L.ptr(left),
                                           L.ptr(r) if right else None, c_size_t(cols)),
            "orbfe_synth_sequence_frame")
    return (left, r) if right else left
