"""ctypes binding of liborbfe.so (include/orbfe.h, orbfe_match_batch.h, orbfe_debug.h, orbfe_synth.h,
orbfe_vocab.h, orbfe_stereo.h, orbfe_frustum.h, orbfe_keyframe.h, orbfe_pack.h, orbfe_c3.h).

The shared library is the product: every compute call below runs the HIP kernels in it. There is
no CPU fallback -- if the library is missing, or no HIP device is present when a compute handle is
created, the call raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, byref, Structure, c_char, c_char_p, c_double, c_float, c_int, c_int32,
                    c_size_t, c_uint8, c_uint32, c_uint64, c_void_p)

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORBFE_LIB", os.path.join(_PKG_DIR, "lib", "liborbfe.so"))

ORBFE_OK = 0
ORBFE_ERR_ARG = -1
ORBFE_ERR_CAPACITY = -2
ORBFE_ERR_HIP = -3
ORBFE_ERR_STATE = -4
ORBFE_RESIZE_SIMD128 = 0
ORBFE_RESIZE_SCALAR = 1
ORBFE_MP_NONE, ORBFE_MP_PRESENT, ORBFE_MP_OBSERVED = 0, 1, 2
ORBFE_MP_BAD = 3  # orbfe_keyframe.h: non-NULL MapPoint with isBad()
MPF_TRACK_IN_VIEW, MPF_BAD, MPF_OBSERVED, MPF_PRESENT, MPF_OUTLIER = 1, 2, 4, 8, 16
MPF_SEEN = 32  # orbfe_frustum.h: mnLastFrameSeen == CurrentFrame.mnId
MPF_SKIP = 64  # orbfe_keyframe.h: already found / in the KeyFrame / already matched

# cv::KeyPoint field order (28 bytes), = orbfe_keypoint
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class OrbfeError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what} failed with status {status}: {last_error()}")
        self.status = status


class LibraryMissing(ImportError):
    pass


class frame_view(Structure):
    _fields_ = [("n", c_int32), ("keys_un", c_void_p), ("u_right", c_void_p),
                ("descriptors", c_void_p), ("mp_state", c_void_p), ("nlevels", c_int32),
                ("scale_factors", c_void_p), ("level_sigma2", c_void_p),
                ("min_x", c_float), ("max_x", c_float), ("min_y", c_float), ("max_y", c_float),
                ("grid_inv_w", c_float), ("grid_inv_h", c_float),
                ("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float),
                ("bf", c_float), ("b", c_float),
                ("grid_origin_set", c_int32), ("grid_min_x", c_float), ("grid_min_y", c_float)]


class feature_vector(Structure):
    _fields_ = [("n_nodes", c_int32), ("node_ids", c_void_p), ("offsets", c_void_p),
                ("indices", c_void_p)]


class local_mappoints(Structure):
    _fields_ = [("m", c_int32), ("flags", c_void_p), ("proj_x", c_void_p), ("proj_y", c_void_p),
                ("proj_xr", c_void_p), ("level", c_void_p), ("view_cos", c_void_p),
                ("descriptors", c_void_p)]


class lastframe_mappoints(Structure):
    _fields_ = [("n", c_int32), ("flags", c_void_p), ("world_pos", c_void_p),
                ("descriptors", c_void_p), ("octave", c_void_p), ("angle", c_void_p),
                ("tcw_last", c_float * 12)]


class mappoint_geometry(Structure):
    _fields_ = [("m", c_int32), ("flags", c_void_p), ("world_pos", c_void_p), ("normal", c_void_p),
                ("min_distance", c_void_p), ("max_distance", c_void_p), ("descriptors", c_void_p)]


class frustum_out(Structure):
    _fields_ = [("flags", c_void_p), ("proj_x", c_void_p), ("proj_y", c_void_p),
                ("proj_xr", c_void_p), ("level", c_void_p), ("view_cos", c_void_p)]


class sft_pair(Structure):
    _fields_ = [("kf1", frame_view), ("kf2", frame_view), ("fv1", feature_vector),
                ("fv2", feature_vector), ("f12", c_float * 9), ("ex", c_float), ("ey", c_float),
                ("match12", c_void_p), ("nmatches", c_void_p), ("kf1_n_dev", c_void_p),
                ("kf2_n_dev", c_void_p), ("fv1_nodes_dev", c_void_p), ("fv2_nodes_dev", c_void_p)]


class c3_set(Structure):  # orbfe_c3.h
    _fields_ = [("kps", c_void_p), ("desc", c_void_p), ("counts", c_void_p), ("fv_node_ids", c_void_p),
                ("fv_offsets", c_void_p), ("fv_indices", c_void_p), ("fv_n_nodes", c_void_p),
                ("bow_words", c_void_p), ("bow_weights", c_void_p), ("bow_n", c_void_p),
                ("u_right", c_void_p), ("depth", c_void_p), ("matcher", c_void_p), ("pairs", c_void_p)]


class c3_config(Structure):
    _fields_ = [("n_images", c_int), ("rows", c_int), ("cols", c_int), ("cap", c_int), ("n_vocab", c_int),
                ("levelsup", c_int), ("n_stereo", c_int), ("mbf", c_float), ("mb", c_float),
                ("stereo_on_match", c_int), ("n_pairs", c_int)]


# name -> (restype, argtypes)
_SIGNATURES = {
    "orbfe_last_error": (c_char_p, []),
    "orbfe_version": (c_char_p, []),
    "orbfe_extractor_create": (c_int, [c_int, c_float, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "orbfe_extractor_destroy": (c_int, [c_void_p]),
    "orbfe_extractor_set_resize_mode": (c_int, [c_void_p, c_int]),
    "orbfe_get_scale_tables": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "orbfe_max_keypoints": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_extract": (c_int, [c_void_p, c_void_p, c_int, c_int, c_size_t, c_void_p, c_int, c_void_p,
                              POINTER(c_int)]),
    "orbfe_extract_batch": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_size_t, c_void_p,
                                    c_void_p, c_int, c_void_p]),
    "orbfe_extract_batch_device": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_int, c_int,
                                           c_size_t, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "orbfe_get_level": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p), POINTER(c_int),
                                POINTER(c_int), POINTER(c_size_t)]),
    "orbfe_get_level_device": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p), POINTER(c_int),
                                       POINTER(c_int), POINTER(c_size_t)]),
    "orbfe_extractor_set_host_pyramid": (c_int, [c_void_p, c_int]),
    "orbfe_extractor_set_graphs": (c_int, [c_void_p, c_int]),
    "orbfe_debug_graph_stats": (c_int, [c_void_p, c_void_p]),
    "orbfe_ktimer_select": (c_int, [ctypes.c_char_p]),
    "orbfe_ktimer_read": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, POINTER(c_int)]),
    "orbfe_ktimer_reset": (c_int, []),
    "orbfe_ktimer_calibrate": (c_int, [c_int, c_int, POINTER(c_double)]),
    "orbfe_extractor_stream": (c_void_p, [c_void_p]),
    "orbfe_extractor_pyramid_event": (c_void_p, [c_void_p]),
    "orbfe_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "orbfe_event_create": (c_int, [c_int, POINTER(c_void_p)]),
    "orbfe_event_record": (c_int, [c_void_p, c_void_p]),
    "orbfe_event_destroy": (c_int, [c_void_p]),
    "orbfe_event_query": (c_int, [c_void_p]),
    "orbfe_matcher_set_profiling": (c_int, [c_void_p, c_int]),
    "orbfe_matcher_last_device_ms": (c_int, [c_void_p, POINTER(c_float)]),
    "orbfe_debug_matcher_sweep_stats": (c_int, [c_void_p, c_void_p]),
    "orbfe_debug_matcher_set_sweep": (c_int, [c_void_p, c_int, c_int, c_int]),
    "orbfe_host_register": (c_int, [c_void_p, c_size_t]),
    "orbfe_host_unregister": (c_int, [c_void_p]),
    "orbfe_stream_create": (c_int, [c_int, c_int, POINTER(c_void_p)]),
    "orbfe_stream_create_masked": (c_int, [c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "orbfe_stream_destroy": (c_int, [c_void_p]),
    "orbfe_matcher_create": (c_int, [c_float, c_int, c_int, POINTER(c_void_p)]),
    "orbfe_matcher_destroy": (c_int, [c_void_p]),
    "orbfe_matcher_stream": (c_void_p, [c_void_p]),
    "orbfe_matcher_last_stats": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    "orbfe_matcher_set_max_rounds": (c_int, [c_void_p, c_int]),
    "orbfe_descriptor_distance": (c_int, [c_void_p, c_void_p]),
    "orbfe_descriptor_distance_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "orbfe_search_by_projection_local": (c_int, [c_void_p, POINTER(frame_view),
                                                 POINTER(local_mappoints), c_float, c_void_p,
                                                 POINTER(c_int)]),
    "orbfe_search_by_projection_lastframe": (c_int, [c_void_p, POINTER(frame_view),
                                                     POINTER(lastframe_mappoints), c_void_p,
                                                     c_float, c_int, c_void_p, POINTER(c_int)]),
    "orbfe_search_for_triangulation": (c_int, [c_void_p, POINTER(frame_view), POINTER(frame_view),
                                               POINTER(feature_vector), POINTER(feature_vector),
                                               c_void_p, c_float, c_float, c_int, c_void_p,
                                               POINTER(c_int)]),
    "orbfe_search_for_triangulation_batch_device": (c_int, [c_void_p, c_int, c_void_p, c_int,
                                                            c_void_p]),
    "orbfe_debug_get_candidates": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, POINTER(c_int)]),
    "orbfe_debug_candidate_total": (c_int, [c_void_p, POINTER(ctypes.c_longlong)]),
    "orbfe_debug_get_level_keys": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, POINTER(c_int)]),
    "orbfe_debug_get_blurred": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int]),
    "orbfe_debug_geometry": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int]),
    "orbfe_debug_set_octree_key_cap": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_fast_side_levels": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_octree_split": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_latency_schedule": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_octree_threads": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_debug_set_octree_threads_l0": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_octree_serial": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_debug_set_pyramid_tiles": (c_int, [c_void_p, c_int, c_int, c_int, c_int]),
    "orbfe_debug_set_zero_copy": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_debug_set_schedule_autotune": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_fast_side_merge": (c_int, [c_void_p, c_int]),
    "orbfe_debug_schedule_choice": (c_int, [c_void_p, c_int]),
    "orbfe_debug_set_octree_lds": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_debug_set_fast_wpb": (c_int, [c_void_p, c_int, c_int]),
    "orbfe_debug_set_inline_side": (c_int, [c_void_p, c_int]),
    "orbfe_set_side_stream": (c_int, [c_void_p, c_void_p]),
    "orbfe_debug_set_blur_mode": (c_int, [c_void_p, c_int]),
    "orbfe_debug_get_umax": (c_int, [c_void_p, c_void_p]),
    "orbfe_debug_steer_trig": (c_int, [c_uint32, c_uint32, c_void_p, c_void_p, c_void_p]),
    "orbfe_vocab_create": (c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_int, POINTER(c_void_p)]),
    "orbfe_vocab_load_text": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "orbfe_vocab_load_binary": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "orbfe_vocab_get_info": (c_int, [c_void_p, c_void_p]),
    "orbfe_vocab_export": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "orbfe_vocab_destroy": (c_int, [c_void_p]),
    # orbfe_pack.h
    "orbfe_packed_bytes": (c_size_t, [c_int, ctypes.c_longlong]),
    "orbfe_pack_keypoints_device": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                            c_size_t, c_void_p, c_void_p]),
    "orbfe_vocab_transform": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                      POINTER(c_int), c_void_p, c_void_p, c_void_p, POINTER(c_int)]),
    "orbfe_vocab_transform_batch_device": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p,
                                                   c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                   c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "orbfe_compute_stereo_matches_batch_device": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p,
                                                          c_void_p, c_void_p, c_int, c_float,
                                                          c_float, c_void_p, c_void_p, c_void_p]),
    "orbfe_compute_stereo_matches": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p,
                                             c_void_p, c_int, c_void_p, c_void_p, c_int, c_float,
                                             c_float, c_void_p, c_void_p]),
    "orbfe_stereo_frame": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_size_t, c_float,
                                   c_float, c_void_p, c_void_p, POINTER(c_int), c_void_p, c_void_p,
                                   POINTER(c_int), c_int, c_void_p, c_void_p]),
    "orbfe_is_in_frustum": (c_int, [c_void_p, POINTER(frame_view), POINTER(mappoint_geometry),
                                    c_void_p, c_float, c_float, POINTER(frustum_out),
                                    POINTER(c_int)]),
    "orbfe_search_local_points": (c_int, [c_void_p, POINTER(frame_view),
                                          POINTER(mappoint_geometry), c_void_p, c_float, c_float,
                                          c_float, c_void_p, POINTER(c_int), POINTER(frustum_out),
                                          POINTER(c_int)]),
    "orbfe_synth_frame": (c_int, [c_uint64, c_int, c_int, c_int, c_void_p, c_void_p, c_size_t]),
    "orbfe_synth_sequence_frame": (c_int, [c_uint64, ctypes.c_longlong, c_int, c_int, c_float, c_float, c_float,
                                           c_float, c_float, c_float, c_void_p, c_void_p, c_size_t]),
    # orbfe_keyframe.h
    "orbfe_search_by_bow_kf_frame": (c_int, [c_void_p, POINTER(frame_view), POINTER(feature_vector),
                                             POINTER(frame_view), POINTER(feature_vector), c_void_p,
                                             POINTER(c_int)]),
    "orbfe_search_by_bow_kf_frame_multi": (c_int, [c_void_p, c_int, c_void_p, c_void_p,
                                                   POINTER(frame_view), POINTER(feature_vector),
                                                   c_void_p, c_void_p]),
    "orbfe_search_by_bow_kf_kf": (c_int, [c_void_p, POINTER(frame_view), POINTER(feature_vector),
                                          POINTER(frame_view), POINTER(feature_vector), c_void_p,
                                          POINTER(c_int)]),
    "orbfe_search_by_projection_keyframe": (c_int, [c_void_p, POINTER(frame_view), c_void_p,
                                                    POINTER(mappoint_geometry), c_void_p, c_float,
                                                    c_float, c_int, c_void_p, POINTER(c_int)]),
    "orbfe_search_by_projection_sim3": (c_int, [c_void_p, POINTER(frame_view), c_void_p,
                                                POINTER(mappoint_geometry), c_float, c_int,
                                                c_void_p, POINTER(c_int)]),
    "orbfe_fuse": (c_int, [c_void_p, POINTER(frame_view), c_void_p, c_void_p,
                           POINTER(mappoint_geometry), c_float, c_float, c_void_p, POINTER(c_int)]),
    "orbfe_fuse_sim3": (c_int, [c_void_p, POINTER(frame_view), c_void_p, POINTER(mappoint_geometry),
                                c_float, c_float, c_void_p, POINTER(c_int)]),
    "orbfe_search_by_sim3": (c_int, [c_void_p, POINTER(frame_view), POINTER(frame_view),
                                     POINTER(mappoint_geometry), POINTER(mappoint_geometry),
                                     c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_float,
                                     c_float, c_float, c_void_p, POINTER(c_int)]),
    "orbfe_search_for_initialization": (c_int, [c_void_p, POINTER(frame_view), POINTER(frame_view),
                                                c_void_p, c_int, c_void_p, POINTER(c_int)]),
    "orbfe_compute_distinctive_descriptors": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "orbfe_compute_distinctive_descriptors_device": (c_int, [c_void_p, c_int, c_void_p, c_void_p,
                                                             c_void_p, c_void_p]),
    "orbfe_predict_scale_thresholds": (c_int, [c_float, c_int, c_void_p]),
    # orbfe_c3.h
    "orbfe_c3_create": (c_int, [POINTER(c3_config), c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                c_void_p, c_int, POINTER(c_void_p)]),
    "orbfe_c3_run": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int]),
    "orbfe_c3_finish": (c_int, [c_void_p, c_int, c_void_p]),
    "orbfe_c3_match_stream": (c_void_p, [c_void_p, c_int]),
    "orbfe_c3_destroy": (c_int, [c_void_p]),
}

# symbols declared in include/*.h (checked by tests/test_library.py)
EXPORTED = sorted(_SIGNATURES)

_lib = None


def lib() -> ctypes.CDLL:
    """Load liborbfe.so once (raises LibraryMissing if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (or make -C orb_slam2_2021_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        ab_build = "ORBFE_LIB" in os.environ  # an A/B build may predate newer entry points
        for name, (res, args) in _SIGNATURES.items():
            if ab_build and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    try:
        s = lib().orbfe_last_error()
    except Exception:  # pragma: no cover
        return "<no library>"
    return s.decode() if s else ""


def check(status: int, what: str) -> int:
    if status < 0:
        raise OrbfeError(status, what)
    return status


def ptr(a) -> c_void_p:
    """Address of a numpy array (contiguous) or an int device pointer."""
    if a is None:
        return c_void_p(0)
    if isinstance(a, int):
        return c_void_p(a)
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):  # torch tensor (device plumbing)
        return c_void_p(a.data_ptr())
    raise TypeError(f"cannot take the address of {type(a)}")


# ---- process-wide kernel timer (orbfe_ktimer_*, include/orbfe.h) ----------------------------------
def ktimer_select(kernels) -> None:
    """Time these kernels' launches by their own dispatch interval (what rocprofv3's kernel trace
    reports): an iterable of names ("k_fast", ...), "*" / True for every kernel, None / False /
    empty for none."""
    if kernels is True:
        v = "*"
    elif not kernels:
        v = ""
    elif isinstance(kernels, str):
        v = kernels
    else:
        v = ",".join(kernels)
    check(lib().orbfe_ktimer_select(v.encode()), "ktimer_select")


def ktimer_read() -> dict:
    """{kernel: (total ms, launches)} of every kernel timed so far (synchronises)."""
    cap, name_len = 64, 48
    names = ctypes.create_string_buffer(cap * name_len)
    total = np.zeros(cap, np.float64)
    launches = np.zeros(cap, np.int64)
    n = c_int()
    check(lib().orbfe_ktimer_read(names, name_len, ptr(total), ptr(launches), cap, ctypes.byref(n)),
          "ktimer_read")
    out = {}
    for k in range(n.value):
        nm = names.raw[k * name_len:(k + 1) * name_len].split(b"\0", 1)[0].decode()
        if launches[k] > 0:
            out[nm] = (float(total[k]), int(launches[k]))
    return out


def ktimer_reset() -> None:
    check(lib().orbfe_ktimer_reset(), "ktimer_reset")


def ktimer_calibrate(device: int = 0, n: int = 64) -> float:
    """The timer's per-dispatch overhead in microseconds (orbfe_ktimer_calibrate)."""
    v = c_double()
    check(lib().orbfe_ktimer_calibrate(int(device), int(n), byref(v)), "ktimer_calibrate")
    return float(v.value)
