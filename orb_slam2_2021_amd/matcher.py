"""ORBmatcher on MI355X -- host mirror of include/ORBmatcher.h over liborbfe.so.

ORBmatcher(nnratio=0.6, checkOri=True) with DescriptorDistance and every search of
include/ORBmatcher.h:41-85. The reference mutates the Frame / KeyFrame / MapPoints it is given;
the mirror returns what it would have written (overloads dispatch on argument types, as in C++):
  SearchByProjection(F, LocalMapPoints, th)             -> (nmatches, best_idx per MapPoint)
  SearchByProjection(F, LastFrameMapPoints, th, bMono)  -> (nmatches, best_idx per last-frame kp)
  SearchByProjection(F, KeyFrame, KeyFrameMapPoints, th, ORBdist) -> (nmatches, best_idx per KF kp)
  SearchByProjection(KeyFrame, Scw, MapPointGeometry, th) -> (nmatches, best_idx per point)
  SearchByBoW(KeyFrame, Frame)     -> (nmatches, KF keypoint per Frame keypoint)
  SearchByBoW(KeyFrame, KeyFrame)  -> (nmatches, KF2 keypoint per KF1 keypoint)
  SearchForInitialization(F1, F2, vbPrevMatched, windowSize) -> (nmatches, vnMatches12, prev)
  SearchForTriangulation(KF1, KF2, F12, bOnlyStereo) -> (nmatches, [(idx1, idx2), ...])
  Fuse(KeyFrame, MapPointGeometry, th) / Fuse(KeyFrame, Scw, MapPointGeometry, th)
                                   -> (count, best_idx per point)
  SearchBySim3(KF1, KF2, mps1, mps2, s12, R12, t12, th) -> (nfound, match12)
  ComputeDistinctiveDescriptors([descriptors per MapPoint]) -> BestIdx per MapPoint
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_void_p
from typing import List, Optional, Tuple, Union

import numpy as np

from . import _lib as L
from .frames import (FeatureVector, Frame, KeyFrame, KeyFrameMapPoints, LastFrameMapPoints,
                     LocalMapPoints, MapPointGeometry, epipole, log_scale_factor)


def _mp_count(mps) -> int:
    """MapPoints of a MapPointGeometry (host arrays) or a DeviceMapPointGeometry."""
    return mps.m if hasattr(mps, "m") else len(mps.flags)


class ORBmatcher:
    TH_HIGH = 100  # ORBmatcher.cc:37-39
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self._lib = L.lib()
        h = c_void_p()
        L.check(self._lib.orbfe_matcher_create(float(nnratio), 1 if checkOri else 0, int(device),
                                               byref(h)), "orbfe_matcher_create")
        self._h = h
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.orbfe_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_profiling(self, on: bool = True) -> None:
        """HIP events around the device part of each host-buffer search (orbfe_matcher_set_profiling)."""
        L.check(self._lib.orbfe_matcher_set_profiling(self._h, 1 if on else 0), "set_profiling")

    def last_device_ms(self) -> float:
        """Device milliseconds of the last profiled search (first to last kernel, no PCIe)."""
        ms = ctypes.c_float()
        L.check(self._lib.orbfe_matcher_last_device_ms(self._h, byref(ms)), "last_device_ms")
        return float(ms.value)

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return L.check(L.lib().orbfe_descriptor_distance(L.ptr(a), L.ptr(b)), "DescriptorDistance")

    def DescriptorDistanceBatch(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        out = np.zeros(len(a), np.int32)
        L.check(self._lib.orbfe_descriptor_distance_batch(self._h, L.ptr(a), L.ptr(b), len(a),
                                                          L.ptr(out)), "distance_batch")
        return out

    def SearchByProjection(self, F: Frame, points, *args, **kw) -> Tuple[int, np.ndarray]:
        """The four overloads of ORBmatcher.h:48-60, by argument types:
        (F, LocalMapPoints, th=3); (F, LastFrameMapPoints, th, bMono);
        (F, KeyFrame, KeyFrameMapPoints, th, ORBdist); (KeyFrame, Scw, MapPointGeometry, th)."""
        if isinstance(points, KeyFrame):
            return self.SearchByProjectionKeyFrame(F, points, *args, **kw)
        if isinstance(F, KeyFrame) and isinstance(points, np.ndarray):
            return self.SearchByProjectionSim3(F, points, *args, **kw)
        th = args[0] if len(args) > 0 else kw.get("th", 3)
        bMono = args[1] if len(args) > 1 else kw.get("bMono")
        return self._search_by_projection_frame(F, points, th, bMono)

    def _search_by_projection_frame(self, F: Frame, points: Union[LocalMapPoints, LastFrameMapPoints],
                                    th: float, bMono: Optional[bool]) -> Tuple[int, np.ndarray]:
        fv = F.view()
        nm = c_int()
        if isinstance(points, LocalMapPoints):
            best = np.full(len(points.flags), -1, np.int32)
            mv = points.view()
            L.check(self._lib.orbfe_search_by_projection_local(self._h, byref(fv), byref(mv),
                                                               float(th), L.ptr(best), byref(nm)),
                    "SearchByProjection(local)")
            return nm.value, best
        if isinstance(points, LastFrameMapPoints):
            if bMono is None:
                raise TypeError("SearchByProjection(CurrentFrame, LastFrame, th, bMono) needs bMono")
            if F.tcw is None:
                raise ValueError("CurrentFrame.tcw (mTcw) is required")
            best = np.full(len(points.flags), -1, np.int32)
            lv = points.view()
            L.check(self._lib.orbfe_search_by_projection_lastframe(
                self._h, byref(fv), byref(lv), L.ptr(F.tcw), float(th), 1 if bMono else 0,
                L.ptr(best), byref(nm)), "SearchByProjection(last frame)")
            return nm.value, best
        raise TypeError("points must be LocalMapPoints or LastFrameMapPoints")

    def SearchByProjectionMotionModel(self, F: Frame, last: LastFrameMapPoints, th: float,
                                      bMono: bool) -> Tuple[int, np.ndarray, float]:
        """Tracking::TrackWithMotionModel's matching (Tracking.cc:896-911): CurrentFrame's
        mvpMapPoints are filled with NULL, SearchByProjection(CurrentFrame, LastFrame, th, bMono)
        runs, and with fewer than 20 matches the map points are cleared again and the search
        repeats at 2 th. F.mp_state is left all ORBFE_MP_NONE (the fill), as the reference's
        Frame is before the caller applies best_idx. Returns (nmatches, best_idx, th used)."""
        F.mp_state = np.zeros(F.N, np.uint8)
        nm, best = self._search_by_projection_frame(F, last, th, bMono)
        if nm < 20:
            th = 2 * th
            nm, best = self._search_by_projection_frame(F, last, th, bMono)
        return nm, best, th

    # ---- Frame::isInFrustum / Tracking::SearchLocalPoints (orbfe_frustum.h) -----------------
    @staticmethod
    def _frustum_out(m: int):
        arrs = {"flags": np.zeros(m, np.uint8), "proj_x": np.zeros(m, np.float32),
                "proj_y": np.zeros(m, np.float32), "proj_xr": np.zeros(m, np.float32),
                "level": np.zeros(m, np.int32), "view_cos": np.zeros(m, np.float32)}
        o = L.frustum_out()
        for k, a in arrs.items():
            setattr(o, k, L.ptr(a))
        return o, arrs

    def isInFrustum(self, F: Frame, mps: MapPointGeometry, viewingCosLimit: float = 0.5,
                    scale_factor: Optional[float] = None) -> Tuple[int, LocalMapPoints]:
        """Frame::isInFrustum (Frame.cc:318-374) for every MapPoint (not BAD, not SEEN) with the
        frame's pose F.tcw. Returns (nToMatch, LocalMapPoints carrying mbTrackInView and the
        mTrackProj* / mnTrackScaleLevel / mTrackViewCos members it writes)."""
        if F.tcw is None:
            raise ValueError("F.tcw (mTcw) is required")
        sf = scale_factor if scale_factor is not None else float(F.scale_factors[1])
        fv, gv = F.view(), mps.view()
        o, arrs = self._frustum_out(_mp_count(mps))
        n = c_int()
        L.check(self._lib.orbfe_is_in_frustum(self._h, byref(fv), byref(gv), L.ptr(F.tcw),
                                              float(log_scale_factor(sf)), float(viewingCosLimit),
                                              byref(o), byref(n)), "isInFrustum")
        return n.value, LocalMapPoints(arrs["flags"], arrs["proj_x"], arrs["proj_y"],
                                       arrs["proj_xr"], arrs["level"], arrs["view_cos"],
                                       mps.descriptors)

    def SearchLocalPoints(self, F: Frame, mps: MapPointGeometry, th: float,
                          viewingCosLimit: float = 0.5, scale_factor: Optional[float] = None
                          ) -> Tuple[int, np.ndarray, int, LocalMapPoints]:
        """Tracking::SearchLocalPoints' projection + matching (Tracking.cc:1186-1213) in one
        device pass: isInFrustum(pMP, 0.5) then SearchByProjection(F, vpLocalMapPoints, th).
        Returns (nmatches, best_idx, nToMatch, LocalMapPoints as isInFrustum left them)."""
        if F.tcw is None:
            raise ValueError("F.tcw (mTcw) is required")
        sf = scale_factor if scale_factor is not None else float(F.scale_factors[1])
        fv, gv = F.view(), mps.view()
        o, arrs = self._frustum_out(_mp_count(mps))
        best = np.full(_mp_count(mps), -1, np.int32)
        nm, nv = c_int(), c_int()
        L.check(self._lib.orbfe_search_local_points(
            self._h, byref(fv), byref(gv), L.ptr(F.tcw), float(log_scale_factor(sf)),
            float(viewingCosLimit), float(th), L.ptr(best), byref(nm), byref(o), byref(nv)),
            "SearchLocalPoints")
        lm = LocalMapPoints(arrs["flags"], arrs["proj_x"], arrs["proj_y"], arrs["proj_xr"],
                            arrs["level"], arrs["view_cos"], mps.descriptors)
        return nm.value, best, nv.value, lm

    def set_max_rounds(self, rounds: int) -> None:
        L.check(self._lib.orbfe_matcher_set_max_rounds(self._h, int(rounds)), "set_max_rounds")

    def last_stats(self) -> Tuple[int, int]:
        r, s = c_int(), c_int()
        L.check(self._lib.orbfe_matcher_last_stats(self._h, byref(r), byref(s)), "last_stats")
        return r.value, s.value

    # ---- keyframe matchers (orbfe_keyframe.h) -----------------------------------------------
    @staticmethod
    def _lsf(F: Frame) -> float:
        sf = float(F.scale_factors[1]) if len(F.scale_factors) > 1 else 1.0
        return float(log_scale_factor(sf))

    def SearchByBoW(self, pKF: KeyFrame, other: Frame) -> Tuple[int, np.ndarray]:
        """SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:165-293) when `other` is a Frame:
        returns (nmatches, KF keypoint index per Frame keypoint or -1).
        SearchByBoW(pKF1, pKF2, vpMatches12) (:536-669) when `other` is a KeyFrame:
        returns (nmatches, KF2 keypoint index per KF1 keypoint or -1)."""
        if pKF.feat_vec is None or other.feat_vec is None:
            raise ValueError("SearchByBoW needs mFeatVec on both sides")
        v1, f1 = pKF.view(), pKF.feat_vec.view()
        v2, f2 = other.view(), other.feat_vec.view()
        nm = c_int()
        if isinstance(other, KeyFrame):
            out = np.full(max(pKF.N, 1), -1, np.int32)
            L.check(self._lib.orbfe_search_by_bow_kf_kf(self._h, byref(v1), byref(f1), byref(v2),
                                                        byref(f2), L.ptr(out), byref(nm)),
                    "SearchByBoW(KF, KF)")
            return nm.value, out[:pKF.N]
        out = np.full(max(other.N, 1), -1, np.int32)
        L.check(self._lib.orbfe_search_by_bow_kf_frame(self._h, byref(v1), byref(f1), byref(v2),
                                                       byref(f2), L.ptr(out), byref(nm)),
                "SearchByBoW(KF, F)")
        return nm.value, out[:other.N]

    def SearchByBoWMulti(self, kfs: List[KeyFrame], F: Frame) -> Tuple[np.ndarray, np.ndarray]:
        """Tracking::Relocalization's SearchByBoW(vpCandidateKFs[i], mCurrentFrame, ...) loop in
        one launch: (nmatches per KF, (n_kf, F.N) KF keypoint per Frame keypoint)."""
        n = len(kfs)
        views = (L.frame_view * max(n, 1))()
        fvs = (L.feature_vector * max(n, 1))()
        for i, kf in enumerate(kfs):
            views[i] = kf.view()
            fvs[i] = kf.feat_vec.view()
        fv, ff = F.view(), F.feat_vec.view()
        out = np.full((max(n, 1), max(F.N, 1)), -1, np.int32)
        counts = np.zeros(max(n, 1), np.int32)
        L.check(self._lib.orbfe_search_by_bow_kf_frame_multi(
            self._h, n, ctypes.addressof(views), ctypes.addressof(fvs), byref(fv), byref(ff),
            L.ptr(out), L.ptr(counts)), "SearchByBoW(KFs, F)")
        return counts[:n], out[:n, :F.N]

    def SearchByProjectionKeyFrame(self, F: Frame, pKF: KeyFrame, pts: KeyFrameMapPoints,
                                   th: float, ORBdist: int) -> Tuple[int, np.ndarray]:
        """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
        (ORBmatcher.cc:1493-1625): best_idx per KF keypoint, encoded as for the last-frame
        overload (k >= 0 assigned, k <= -2 assigned then undone by the rotation filter)."""
        if F.tcw is None:
            raise ValueError("CurrentFrame.tcw (mTcw) is required")
        fv, gv = F.view(), pts.geometry.view()
        best = np.full(max(len(pts.angle), 1), -1, np.int32)
        nm = c_int()
        L.check(self._lib.orbfe_search_by_projection_keyframe(
            self._h, byref(fv), L.ptr(F.tcw), byref(gv), L.ptr(pts.angle), self._lsf(F), float(th),
            int(ORBdist), L.ptr(best), byref(nm)), "SearchByProjection(F, KF)")
        return nm.value, best[:len(pts.angle)]

    def SearchByProjectionSim3(self, pKF: KeyFrame, Scw: np.ndarray, pts: MapPointGeometry,
                               th: int) -> Tuple[int, np.ndarray]:
        """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:295-412);
        pKF.mp_state encodes vpMatched. best_idx[i] = keypoint for vpPoints[i] or -1."""
        kv, gv = pKF.view(), pts.view()
        scw = np.ascontiguousarray(np.asarray(Scw, np.float32).reshape(-1, 4)[:3], np.float32)
        best = np.full(max(len(pts.flags), 1), -1, np.int32)
        nm = c_int()
        L.check(self._lib.orbfe_search_by_projection_sim3(
            self._h, byref(kv), L.ptr(scw), byref(gv), self._lsf(pKF), int(th), L.ptr(best),
            byref(nm)), "SearchByProjection(KF, Scw)")
        return nm.value, best[:len(pts.flags)]

    def Fuse(self, pKF: KeyFrame, *args) -> Tuple[int, np.ndarray]:
        """Fuse(pKF, vpMapPoints, th=3.0) (ORBmatcher.cc:841-991) or Fuse(pKF, Scw, vpPoints, th)
        (:993-1120): the keypoint each MapPoint is fused into (or -1). For the first overload the
        count is the number of candidates (the adapter re-tests isBad / IsInKeyFrame as it
        applies them); for the Scw overload it is the reference's return value."""
        kv = pKF.view()
        if len(args) and isinstance(args[0], np.ndarray) and args[0].size in (12, 16):
            scw = np.ascontiguousarray(np.asarray(args[0], np.float32).reshape(-1, 4)[:3])
            pts, th = args[1], float(args[2])
            gv = pts.view()
            best = np.full(max(len(pts.flags), 1), -1, np.int32)
            n = c_int()
            L.check(self._lib.orbfe_fuse_sim3(self._h, byref(kv), L.ptr(scw), byref(gv),
                                              self._lsf(pKF), th, L.ptr(best), byref(n)),
                    "Fuse(KF, Scw)")
            return n.value, best[:len(pts.flags)]
        pts = args[0]
        th = float(args[1]) if len(args) > 1 else 3.0
        if pKF.tcw is None:
            raise ValueError("pKF.tcw (GetPose) is required")
        gv = pts.view()
        ow = pKF.camera_center
        best = np.full(max(len(pts.flags), 1), -1, np.int32)
        n = c_int()
        L.check(self._lib.orbfe_fuse(self._h, byref(kv), L.ptr(pKF.tcw), L.ptr(ow), byref(gv),
                                     self._lsf(pKF), th, L.ptr(best), byref(n)), "Fuse(KF)")
        return n.value, best[:len(pts.flags)]

    def SearchBySim3(self, pKF1: KeyFrame, pKF2: KeyFrame, mps1: MapPointGeometry,
                     mps2: MapPointGeometry, s12: float, R12: np.ndarray, t12: np.ndarray,
                     th: float) -> Tuple[int, np.ndarray]:
        """SearchBySim3 (ORBmatcher.cc:1122-1346): (nFound, KF2 keypoint per KF1 keypoint where
        both directions agree, else -1). mps1 / mps2 flags: MPF_PRESENT, MPF_BAD, MPF_SKIP
        (vbAlreadyMatched)."""
        v1, v2, g1, g2 = pKF1.view(), pKF2.view(), mps1.view(), mps2.view()
        r12 = np.ascontiguousarray(R12, np.float32).reshape(9)
        t = np.ascontiguousarray(t12, np.float32).reshape(3)
        out = np.full(max(pKF1.N, 1), -1, np.int32)
        n = c_int()
        L.check(self._lib.orbfe_search_by_sim3(
            self._h, byref(v1), byref(v2), byref(g1), byref(g2), L.ptr(pKF1.tcw), L.ptr(pKF2.tcw),
            float(s12), L.ptr(r12), L.ptr(t), self._lsf(pKF1), self._lsf(pKF2), float(th),
            L.ptr(out), byref(n)), "SearchBySim3")
        return n.value, out[:pKF1.N]

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray,
                                windowSize: int = 10) -> Tuple[int, np.ndarray, np.ndarray]:
        """SearchForInitialization (ORBmatcher.cc:414-534): (nmatches, vnMatches12, updated
        vbPrevMatched as an (N1, 2) float32 array)."""
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).reshape(F1.N, 2).copy()
        v1, v2 = F1.view(), F2.view()
        out = np.full(max(F1.N, 1), -1, np.int32)
        nm = c_int()
        L.check(self._lib.orbfe_search_for_initialization(self._h, byref(v1), byref(v2), L.ptr(prev),
                                                          int(windowSize), L.ptr(out), byref(nm)),
                "SearchForInitialization")
        return nm.value, out[:F1.N], prev

    def ComputeDistinctiveDescriptors(self, descriptor_sets: List[np.ndarray]) -> np.ndarray:
        """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:272-337) for many MapPoints at
        once: BestIdx into each MapPoint's (n_i, 32) descriptor rows (-1 when n_i == 0)."""
        counts = np.array([len(d) for d in descriptor_sets], np.int64)
        offsets = np.zeros(len(descriptor_sets) + 1, np.int32)
        offsets[1:] = np.cumsum(counts)
        desc = (np.ascontiguousarray(np.concatenate([np.asarray(d, np.uint8).reshape(-1, 32)
                                                     for d in descriptor_sets]), np.uint8)
                if len(descriptor_sets) and offsets[-1] else np.zeros((1, 32), np.uint8))
        out = np.full(max(len(descriptor_sets), 1), -1, np.int32)
        L.check(self._lib.orbfe_compute_distinctive_descriptors(
            self._h, len(descriptor_sets), L.ptr(offsets), L.ptr(desc), L.ptr(out)),
            "ComputeDistinctiveDescriptors")
        return out[:len(descriptor_sets)]

    def SearchForTriangulation(self, pKF1: Frame, pKF2: Frame, F12: np.ndarray,
                               bOnlyStereo: bool = False,
                               epipole_xy: Optional[Tuple[float, float]] = None
                               ) -> Tuple[int, List[Tuple[int, int]], np.ndarray]:
        if pKF1.feat_vec is None or pKF2.feat_vec is None:
            raise ValueError("KeyFrames need feat_vec (mFeatVec)")
        ex, ey = epipole_xy if epipole_xy is not None else epipole(pKF1, pKF2)
        f12 = np.ascontiguousarray(F12, np.float32).reshape(9)
        v1, v2 = pKF1.view(), pKF2.view()
        fv1, fv2 = pKF1.feat_vec.view(), pKF2.feat_vec.view()
        m12 = np.full(max(pKF1.N, 1), -1, np.int32)
        nm = c_int()
        L.check(self._lib.orbfe_search_for_triangulation(
            self._h, byref(v1), byref(v2), byref(fv1), byref(fv2), L.ptr(f12), float(ex), float(ey),
            1 if bOnlyStereo else 0, L.ptr(m12), byref(nm)), "SearchForTriangulation")
        m12 = m12[:pKF1.N]
        pairs = [(int(i), int(m12[i])) for i in np.nonzero(m12 >= 0)[0]]
        return nm.value, pairs, m12
