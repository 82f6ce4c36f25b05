"""ORBmatcher on MI355X -- host mirror of include/ORBmatcher.h over liborbfe.so.

ORBmatcher(nnratio=0.6, checkOri=True) with DescriptorDistance, both SearchByProjection overloads
used by Tracking and SearchForTriangulation used by LocalMapping (include/ORBmatcher.h:41-85).
The reference mutates the Frame it is given; the mirror returns what it would have written:
  SearchByProjection(F, LocalMapPoints, th)      -> (nmatches, best_idx per MapPoint)
  SearchByProjection(F, LastFrameMapPoints, th, bMono) -> (nmatches, best_idx per last-frame kp)
  SearchForTriangulation(KF1, KF2, F12, bOnlyStereo) -> (nmatches, [(idx1, idx2), ...])
"""
from __future__ import annotations

from ctypes import byref, c_int, c_void_p
from typing import List, Optional, Tuple, Union

import numpy as np

from . import _lib as L
from .frames import (FeatureVector, Frame, LastFrameMapPoints, LocalMapPoints, MapPointGeometry,
                     epipole, log_scale_factor)


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

    def SearchByProjection(self, F: Frame, points: Union[LocalMapPoints, LastFrameMapPoints],
                           th: float = 3, bMono: Optional[bool] = None) -> Tuple[int, np.ndarray]:
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
        o, arrs = self._frustum_out(len(mps.flags))
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
        o, arrs = self._frustum_out(len(mps.flags))
        best = np.full(len(mps.flags), -1, np.int32)
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
