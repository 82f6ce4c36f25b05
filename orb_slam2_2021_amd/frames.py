"""Packed views of the ORB-SLAM2 objects the matchers read (host-side mirror of the reference).

ORBmatcher reads Frame / KeyFrame / MapPoint state through pointers and mutexes
(ORBmatcher.cc:45-133, 671-839, 1348-1491). The drop-in boundary takes them as struct-of-arrays
(include/orbfe.h); these dataclasses hold those arrays and produce the C structs.
Field names follow the reference members they stand for.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L

FRAME_GRID_ROWS = 48  # Frame.h:38
FRAME_GRID_COLS = 64  # Frame.h:39


def _f32(x) -> np.float32:
    return np.float32(x)


@dataclass
class Frame:
    """Frame / KeyFrame fields used by SearchByProjection and SearchForTriangulation."""

    keys_un: np.ndarray            # mvKeysUn, KEYPOINT_DTYPE
    descriptors: np.ndarray        # mDescriptors, (N, 32) uint8
    u_right: np.ndarray            # mvuRight, float32 (-1 = no stereo match)
    mp_state: np.ndarray           # ORBFE_MP_* per keypoint (mvpMapPoints / GetMapPoint)
    scale_factors: np.ndarray      # mvScaleFactors
    level_sigma2: np.ndarray       # mvLevelSigma2
    min_x: float = 0.0             # mnMinX ... (Frame.cc:515-518 for undistorted images)
    max_x: float = 0.0
    min_y: float = 0.0
    max_y: float = 0.0
    fx: float = 0.0
    fy: float = 0.0
    cx: float = 0.0
    cy: float = 0.0
    bf: float = 0.0                # mbf
    tcw: Optional[np.ndarray] = None          # mTcw rows 0..2 (3x4 float32)
    feat_vec: Optional["FeatureVector"] = None  # mFeatVec (KeyFrame)

    def __post_init__(self):
        self.keys_un = np.ascontiguousarray(self.keys_un, dtype=L.KEYPOINT_DTYPE)
        n = len(self.keys_un)
        self.descriptors = np.ascontiguousarray(self.descriptors, dtype=np.uint8).reshape(n, 32)
        self.u_right = np.ascontiguousarray(self.u_right, dtype=np.float32).reshape(n)
        self.mp_state = np.ascontiguousarray(self.mp_state, dtype=np.uint8).reshape(n)
        self.scale_factors = np.ascontiguousarray(self.scale_factors, dtype=np.float32)
        self.level_sigma2 = np.ascontiguousarray(self.level_sigma2, dtype=np.float32)
        if self.tcw is not None:
            self.tcw = np.ascontiguousarray(self.tcw, dtype=np.float32).reshape(3, 4)

    @property
    def N(self) -> int:
        return len(self.keys_un)

    @property
    def grid_inv_w(self) -> np.float32:
        # mfGridElementWidthInv = float(FRAME_GRID_COLS) / (mnMaxX - mnMinX)  (Frame.cc:136)
        return _f32(FRAME_GRID_COLS) / (_f32(self.max_x) - _f32(self.min_x))

    @property
    def grid_inv_h(self) -> np.float32:
        return _f32(FRAME_GRID_ROWS) / (_f32(self.max_y) - _f32(self.min_y))

    @property
    def mb(self) -> np.float32:
        return _f32(self.bf) / _f32(self.fx) if self.fx else _f32(0.0)

    def view(self) -> L.frame_view:
        v = L.frame_view()
        v.n = self.N
        v.keys_un = L.ptr(self.keys_un)
        v.u_right = L.ptr(self.u_right)
        v.descriptors = L.ptr(self.descriptors)
        v.mp_state = L.ptr(self.mp_state)
        v.nlevels = len(self.scale_factors)
        v.scale_factors = L.ptr(self.scale_factors)
        v.level_sigma2 = L.ptr(self.level_sigma2)
        v.min_x, v.max_x, v.min_y, v.max_y = self.min_x, self.max_x, self.min_y, self.max_y
        v.grid_inv_w, v.grid_inv_h = float(self.grid_inv_w), float(self.grid_inv_h)
        v.fx, v.fy, v.cx, v.cy, v.bf = self.fx, self.fy, self.cx, self.cy, self.bf
        v.b = float(self.mb)
        return v


class KeyFrame(Frame):
    """KeyFrame(F, pMap, pKFDB) as the keyframe matchers read it (KeyFrame.cc:29-64): the Frame's
    keypoints, descriptors and tables, with the image bounds narrowed to the KeyFrame's
    `const int` mnMinX.. (KeyFrame.h:202-205) while mGrid stays the Frame's grid (built with the
    Frame's float bounds and cell sizes). mp_state is GetMapPointMatches() (ORBFE_MP_BAD for a
    MapPoint with isBad())."""

    grid_origin: Optional[tuple] = None  # the Frame's (mnMinX, mnMinY) that built mGrid
    grid_inv: Optional[tuple] = None     # the Frame's (mfGridElementWidthInv, ...HeightInv)

    @staticmethod
    def from_frame(F: "Frame", tcw: Optional[np.ndarray] = None,
                   mp_state: Optional[np.ndarray] = None) -> "KeyFrame":
        kf = KeyFrame(keys_un=F.keys_un, descriptors=F.descriptors, u_right=F.u_right,
                      mp_state=F.mp_state if mp_state is None else mp_state,
                      scale_factors=F.scale_factors, level_sigma2=F.level_sigma2,
                      min_x=float(int(F.min_x)), max_x=float(int(F.max_x)),
                      min_y=float(int(F.min_y)), max_y=float(int(F.max_y)),
                      fx=F.fx, fy=F.fy, cx=F.cx, cy=F.cy, bf=F.bf,
                      tcw=F.tcw if tcw is None else tcw, feat_vec=F.feat_vec)
        kf.grid_origin = (float(F.min_x), float(F.min_y))
        kf.grid_inv = (float(F.grid_inv_w), float(F.grid_inv_h))
        return kf

    @property
    def grid_inv_w(self) -> np.float32:
        return _f32(self.grid_inv[0]) if self.grid_inv else Frame.grid_inv_w.fget(self)

    @property
    def grid_inv_h(self) -> np.float32:
        return _f32(self.grid_inv[1]) if self.grid_inv else Frame.grid_inv_h.fget(self)

    @property
    def camera_center(self) -> np.ndarray:
        """GetCameraCenter(): Ow = -Rcw^T tcw (gemm, double accumulation)."""
        R, t = self.tcw[:, :3], self.tcw[:, 3]
        return np.array([-gemv_f32_double(R.T[i:i + 1], t)[0] for i in range(3)], np.float32)

    def view(self) -> L.frame_view:
        v = Frame.view(self)
        if self.grid_origin is not None:
            v.grid_origin_set = 1
            v.grid_min_x, v.grid_min_y = self.grid_origin
        return v


@dataclass
class FeatureVector:
    """DBoW2::FeatureVector (node id -> ascending feature indices) as CSR."""

    node_ids: np.ndarray  # uint32, ascending
    offsets: np.ndarray   # int32, len n_nodes + 1
    indices: np.ndarray   # int32

    @staticmethod
    def from_assignment(node_of_feature: Sequence[int]) -> "FeatureVector":
        """Features pushed in index order into their node's list (TemplatedVocabulary.h:1161-1174)."""
        node_of_feature = np.asarray(node_of_feature, dtype=np.int64)
        order = np.argsort(node_of_feature, kind="stable")
        nodes = node_of_feature[order]
        ids, starts = np.unique(nodes, return_index=True)
        offsets = np.append(starts, len(nodes)).astype(np.int32)
        return FeatureVector(ids.astype(np.uint32), offsets, order.astype(np.int32))

    @staticmethod
    def from_dict(d: Dict[int, List[int]]) -> "FeatureVector":
        ids = sorted(d)
        offs = [0]
        idx: List[int] = []
        for k in ids:
            idx.extend(d[k])
            offs.append(len(idx))
        return FeatureVector(np.array(ids, np.uint32), np.array(offs, np.int32),
                             np.array(idx, np.int32))

    def __post_init__(self):
        self.node_ids = np.ascontiguousarray(self.node_ids, dtype=np.uint32)
        self.offsets = np.ascontiguousarray(self.offsets, dtype=np.int32)
        self.indices = np.ascontiguousarray(self.indices, dtype=np.int32)

    def view(self) -> L.feature_vector:
        v = L.feature_vector()
        v.n_nodes = len(self.node_ids)
        v.node_ids = L.ptr(self.node_ids)
        v.offsets = L.ptr(self.offsets)
        v.indices = L.ptr(self.indices) if len(self.indices) else L.ptr(np.zeros(1, np.int32))
        return v


@dataclass
class LocalMapPoints:
    """Local-map MapPoints after Frame::isInFrustum (Frame.cc:366-371)."""

    flags: np.ndarray        # MPF_TRACK_IN_VIEW | MPF_BAD | MPF_OBSERVED
    proj_x: np.ndarray       # mTrackProjX
    proj_y: np.ndarray       # mTrackProjY
    proj_xr: np.ndarray      # mTrackProjXR
    level: np.ndarray        # mnTrackScaleLevel
    view_cos: np.ndarray     # mTrackViewCos
    descriptors: np.ndarray  # GetDescriptor()

    def __post_init__(self):
        m = len(self.flags)
        self.flags = np.ascontiguousarray(self.flags, np.uint8)
        self.proj_x = np.ascontiguousarray(self.proj_x, np.float32).reshape(m)
        self.proj_y = np.ascontiguousarray(self.proj_y, np.float32).reshape(m)
        self.proj_xr = np.ascontiguousarray(self.proj_xr, np.float32).reshape(m)
        self.level = np.ascontiguousarray(self.level, np.int32).reshape(m)
        self.view_cos = np.ascontiguousarray(self.view_cos, np.float32).reshape(m)
        if not getattr(self.descriptors, "is_cuda", False):  # a resident map's stay on the device
            self.descriptors = np.ascontiguousarray(self.descriptors, np.uint8).reshape(m, 32)

    def view(self) -> L.local_mappoints:
        v = L.local_mappoints()
        v.m = len(self.flags)
        for f in ("flags", "proj_x", "proj_y", "proj_xr", "level", "view_cos", "descriptors"):
            setattr(v, f, L.ptr(getattr(self, f)))
        return v


@dataclass
class MapPointGeometry:
    """Local-map MapPoints as Frame::isInFrustum reads them (Frame.cc:318-374)."""

    flags: np.ndarray         # MPF_BAD | MPF_SEEN (| MPF_OBSERVED, passed to SearchByProjection)
    world_pos: np.ndarray     # (M, 3) GetWorldPos()
    normal: np.ndarray        # (M, 3) GetNormal()
    min_distance: np.ndarray  # mfMinDistance
    max_distance: np.ndarray  # mfMaxDistance
    descriptors: np.ndarray   # (M, 32) GetDescriptor()

    def __post_init__(self):
        m = len(self.flags)
        self.flags = np.ascontiguousarray(self.flags, np.uint8)
        self.world_pos = np.ascontiguousarray(self.world_pos, np.float32).reshape(m, 3)
        self.normal = np.ascontiguousarray(self.normal, np.float32).reshape(m, 3)
        self.min_distance = np.ascontiguousarray(self.min_distance, np.float32).reshape(m)
        self.max_distance = np.ascontiguousarray(self.max_distance, np.float32).reshape(m)
        self.descriptors = np.ascontiguousarray(self.descriptors, np.uint8).reshape(m, 32)

    def view(self) -> L.mappoint_geometry:
        v = L.mappoint_geometry()
        v.m = len(self.flags)
        for f in ("flags", "world_pos", "normal", "min_distance", "max_distance", "descriptors"):
            setattr(v, f, L.ptr(getattr(self, f)))
        return v


class DeviceMapPointGeometry:
    """A MapPointGeometry resident in HBM (C5's replicated local map, uploaded or broadcast once):
    the same SoA fields as contiguous device tensors (any dtype: the bytes are what count). The
    matcher copies device inputs on the device instead of staging them through the host
    (orbfe_frustum.h). Built from a MapPointGeometry and a torch device, or from tensors already
    on the device (parallel.broadcast_arrays' output)."""

    FIELDS = ("flags", "world_pos", "normal", "min_distance", "max_distance", "descriptors")

    def __init__(self, geometry: Optional["MapPointGeometry"] = None, device=None, tensors=None, m=None):
        import torch
        if tensors is None:
            tensors = {f: torch.from_numpy(np.ascontiguousarray(getattr(geometry, f))).to(device)
                       for f in self.FIELDS}
            m = len(geometry.flags)
        if m is None:
            raise ValueError("m (the MapPoint count) is required with tensors")
        for f in self.FIELDS:
            t = tensors[f]
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError(f"{f}: a contiguous device tensor is required")
            setattr(self, f, t)
        self.m = int(m)
        # the matcher reads these on its own non-blocking stream, which nothing orders after the
        # stream that wrote them (torch's current stream: the upload, or RCCL's broadcast into them,
        # parallel.broadcast_arrays): wait for that writer here, once, before any search uses the map
        torch.cuda.current_stream(self.flags.device).synchronize()
        need = {"flags": 1, "world_pos": 12, "normal": 12, "min_distance": 4, "max_distance": 4, "descriptors": 32}
        for f, b in need.items():
            if getattr(self, f).numel() * getattr(self, f).element_size() < b * self.m:
                raise ValueError(f"{f}: fewer than {b} bytes per MapPoint")

    def __len__(self) -> int:
        return self.m

    def view(self) -> L.mappoint_geometry:
        v = L.mappoint_geometry()
        v.m = self.m
        for f in self.FIELDS:
            setattr(v, f, L.ptr(getattr(self, f).data_ptr()))
        return v


@dataclass
class KeyFrameMapPoints:
    """pKF->GetMapPointMatches() by KeyFrame keypoint with the KeyFrame's mvKeysUn angles, as
    SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) reads them
    (ORBmatcher.cc:1511-1595). geometry.flags: MPF_PRESENT, MPF_BAD, MPF_SKIP (in sAlreadyFound)."""

    geometry: MapPointGeometry
    angle: np.ndarray

    def __post_init__(self):
        self.angle = np.ascontiguousarray(self.angle, np.float32).reshape(len(self.geometry.flags))


_libm = None


def log_scale_factor(scale_factor: float) -> np.float32:
    """Frame::mfLogScaleFactor = log(mfScaleFactor) (Frame.cc:106). mfScaleFactor is a float and
    the translation unit sees `using namespace std` (TemplatedVocabulary.h:36), so this is the
    float overload: the C library's logf."""
    global _libm
    if _libm is None:
        import ctypes
        import ctypes.util
        _libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _libm.logf.restype = ctypes.c_float
        _libm.logf.argtypes = [ctypes.c_float]
    return np.float32(_libm.logf(float(np.float32(scale_factor))))


@dataclass
class LastFrameMapPoints:
    """LastFrame.mvpMapPoints and the per-keypoint data SearchByProjection reads from it."""

    flags: np.ndarray        # MPF_PRESENT | MPF_OUTLIER | MPF_OBSERVED
    world_pos: np.ndarray    # (N, 3) GetWorldPos()
    descriptors: np.ndarray  # (N, 32) GetDescriptor()
    octave: np.ndarray       # LastFrame.mvKeys[i].octave
    angle: np.ndarray        # LastFrame.mvKeysUn[i].angle
    tcw_last: np.ndarray     # LastFrame.mTcw rows 0..2

    def __post_init__(self):
        n = len(self.flags)
        self.flags = np.ascontiguousarray(self.flags, np.uint8)
        self.world_pos = np.ascontiguousarray(self.world_pos, np.float32).reshape(n, 3)
        self.descriptors = np.ascontiguousarray(self.descriptors, np.uint8).reshape(n, 32)
        self.octave = np.ascontiguousarray(self.octave, np.int32).reshape(n)
        self.angle = np.ascontiguousarray(self.angle, np.float32).reshape(n)
        self.tcw_last = np.ascontiguousarray(self.tcw_last, np.float32).reshape(3, 4)

    def view(self) -> L.lastframe_mappoints:
        v = L.lastframe_mappoints()
        v.n = len(self.flags)
        for f in ("flags", "world_pos", "descriptors", "octave", "angle"):
            setattr(v, f, L.ptr(getattr(self, f)))
        for i, x in enumerate(self.tcw_last.reshape(12)):
            v.tcw_last[i] = float(x)
        return v


def gemv_f32_double(A: np.ndarray, x: np.ndarray, add: Optional[np.ndarray] = None) -> np.ndarray:
    """cv::Mat CV_32F A*x (+ add): products and sums in double, one rounding to float
    (SURVEY Appendix A.9)."""
    A = np.asarray(A, np.float32)
    x = np.asarray(x, np.float32)
    out = np.empty(A.shape[0], np.float32)
    for r in range(A.shape[0]):
        s = float(np.float64(A[r, 0]) * np.float64(x[0]))
        for k in range(1, A.shape[1]):
            s = s + float(np.float64(A[r, k]) * np.float64(x[k]))
        if add is not None:
            s = s + float(np.float64(np.float32(add[r])))
        out[r] = np.float32(s)
    return out


def camera_center(tcw: np.ndarray) -> np.ndarray:
    """KeyFrame::GetCameraCenter: Ow = -Rcw^T * tcw."""
    tcw = np.asarray(tcw, np.float32).reshape(3, 4)
    return -gemv_f32_double(tcw[:, :3].T.copy(), tcw[:, 3])


def epipole(kf1: Frame, kf2: Frame):
    """(ex, ey) of KF1's centre in KF2 (ORBmatcher.cc:677-684)."""
    Cw = camera_center(kf1.tcw)
    C2 = gemv_f32_double(kf2.tcw[:, :3], Cw, kf2.tcw[:, 3])
    invz = np.float32(1.0) / C2[2]
    ex = np.float32(kf2.fx) * C2[0] * invz + np.float32(kf2.cx)
    ey = np.float32(kf2.fy) * C2[1] * invz + np.float32(kf2.cy)
    return float(ex), float(ey)
