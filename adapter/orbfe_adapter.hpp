/*
 * orbfe_adapter.hpp -- the bodies of the GPU build's ORBmatcher methods (adapter/ORBmatcher_gpu.cc)
 * as templates over the matcher facade `M` (orbfe::Matcher, include/orbfe.hpp) and the reference's
 * Frame / KeyFrame / MapPoint types: pack (orbfe_pack.hpp), search on the GPU, apply the result
 * to the object graph in the reference's loop order. ORBmatcher_gpu.cc instantiates them on the
 * real classes; tests/cpp/adapter_pack_test.cpp instantiates every one on Frame-shaped test
 * structs with a recording matcher, so the packing and the application are checked on the CPU.
 *
 * Each function cites the reference method it stands in for (src/ORBmatcher.cc). What the search
 * itself computes is liborbfe's (bit-exact with the oracle, tests/test_gpu_match.py and
 * tests/test_gpu_keyframe.py); here only what the reference does around it.
 */
#ifndef ORBFE_ADAPTER_HPP
#define ORBFE_ADAPTER_HPP

#include <set>
#include <type_traits>
#include <utility>
#include <vector>

#include "orbfe_pack.hpp"

namespace orbfe_adapter {

template <class KF>
using mp_of_t = typename std::remove_pointer<typename decltype(std::declval<KF&>().GetMapPointMatches())::value_type>::type;

// SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, th) (:45-133)
template <class M, class F, class MP>
int search_by_projection_local(M& m, F& f, const std::vector<MP*>& vpMapPoints, float th) {
  FramePack pf;
  pack_frame(f, f.mvpMapPoints, pf);
  LocalMapPack lp(vpMapPoints);
  std::vector<int32_t> best;
  const int n = m.SearchByProjection(pf.v, lp.view(), th, best);
  apply_local_matches(best, f.mvpMapPoints, vpMapPoints);
  return n;
}

// SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) (:1348-1491)
template <class M, class F>
int search_by_projection_lastframe(M& m, F& cur, const F& last, float th, bool mono) {
  FramePack pc;
  pack_frame(cur, cur.mvpMapPoints, pc);
  LastFramePack lp(last);
  std::vector<int32_t> best;
  const int n = m.SearchByProjection(pc.v, lp.view(), mat_floats(cur.mTcw), th, mono, best);
  apply_lastframe_matches(best, cur.mvpMapPoints, last.mvpMapPoints);
  return n;
}

// SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) (:671-839). f12: F12 as a
// continuous 3x3 CV_32F; (ex, ey): the epipole, computed by the caller with the reference's own
// cv::Mat expression (:678-684)
template <class M, class KF, class Pairs>
int search_for_triangulation(M& m, KF* k1, KF* k2, const float* f12, float ex, float ey, Pairs& pairs,
                             bool only_stereo) {
  FramePack p1, p2;
  pack_frame(*k1, k1->GetMapPointMatches(), p1);
  pack_frame(*k2, k2->GetMapPointMatches(), p2);
  CsrFeatureVector fv1(k1->mFeatVec), fv2(k2->mFeatVec);
  return m.SearchForTriangulation(p1.v, p2.v, fv1.view(), fv2.view(), f12, ex, ey, pairs, only_stereo);
}

// SearchByBoW(pKF, F, vpMapPointMatches) (:165-293)
template <class M, class KF, class F, class MP>
int search_by_bow(M& m, KF* kf, F& f, std::vector<MP*>& vpMapPointMatches, float gx, float gy) {
  FramePack pk, pf;
  pack_keyframe(*kf, pk, gx, gy);
  pack_frame(f, f.mvpMapPoints, pf);  // the Frame's MapPoints are not read
  CsrFeatureVector fk(kf->mFeatVec), ff(f.mFeatVec);
  std::vector<int32_t> kf_of_f;
  const int n = m.SearchByBoW(pk.v, fk.view(), pf.v, ff.view(), kf_of_f);
  const std::vector<MP*> mpsKF = kf->GetMapPointMatches();
  vpMapPointMatches.assign(f.N, nullptr);
  for (int k = 0; k < f.N; k++)
    if (kf_of_f[k] >= 0) vpMapPointMatches[k] = mpsKF[kf_of_f[k]];
  return n;
}

// SearchByBoW(pKF1, pKF2, vpMatches12) (:536-669)
template <class M, class KF, class MP>
int search_by_bow12(M& m, KF* k1, KF* k2, std::vector<MP*>& vpMatches12, float gx, float gy) {
  FramePack p1, p2;
  pack_keyframe(*k1, p1, gx, gy);
  pack_keyframe(*k2, p2, gx, gy);
  CsrFeatureVector f1(k1->mFeatVec), f2(k2->mFeatVec);
  std::vector<int32_t> m12;
  const int n = m.SearchByBoW12(p1.v, f1.view(), p2.v, f2.view(), m12);
  const std::vector<MP*> mps2 = k2->GetMapPointMatches();
  vpMatches12.assign(k1->N, nullptr);
  for (int i = 0; i < k1->N; i++)
    if (m12[i] >= 0) vpMatches12[i] = mps2[m12[i]];
  return n;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1493-1625)
template <class M, class F, class KF, class Set, class DistOf>
int search_by_projection_keyframe(M& m, F& cur, KF* kf, const Set& sAlreadyFound, float th, int orb_dist,
                                  DistOf dist_of) {
  using MP = mp_of_t<KF>;
  FramePack pc;
  pack_frame(cur, cur.mvpMapPoints, pc);  // any non-NULL entry is taken
  const std::vector<MP*> mps = kf->GetMapPointMatches();
  GeometryPack g(mps, [&](MP* p) -> unsigned {
    return ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u) | (sAlreadyFound.count(p) ? ORBFE_MPF_SKIP : 0u);
  }, dist_of);
  std::vector<float> angle(kf->N);
  for (int i = 0; i < kf->N; i++) angle[i] = kf->mvKeysUn[i].angle;
  std::vector<int32_t> best;
  const int n = m.SearchByProjection(pc.v, mat_floats(cur.mTcw), g.view(), angle.data(), cur.mfLogScaleFactor, th,
                                     orb_dist, best);
  apply_lastframe_matches(best, cur.mvpMapPoints, mps);
  return n;
}

// SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (:295-412); scw: Scw continuous 4x4 CV_32F
template <class M, class KF, class MP, class DistOf>
int search_by_projection_sim3(M& m, KF* kf, const float* scw, const std::vector<MP*>& vpPoints,
                              std::vector<MP*>& vpMatched, int th, DistOf dist_of, float gx, float gy) {
  FramePack pk;
  pack_keyframe(*kf, pk, gx, gy);
  for (int i = 0; i < kf->N; i++) pk.mp_state[i] = vpMatched[i] ? ORBFE_MP_PRESENT : ORBFE_MP_NONE;
  std::set<MP*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
  spAlreadyFound.erase(static_cast<MP*>(nullptr));
  GeometryPack g(vpPoints, [&](MP* p) -> unsigned {
    return ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u) | (spAlreadyFound.count(p) ? ORBFE_MPF_SKIP : 0u);
  }, dist_of);
  std::vector<int32_t> best;
  const int n = m.SearchByProjectionSim3(pk.v, scw, g.view(), kf->mfLogScaleFactor, th, best);
  apply_local_matches(best, vpMatched, vpPoints);
  return n;
}

// Fuse(pKF, vpMapPoints, th) (:841-991): the search, then the reference's own replace / add in
// ascending order, re-testing isBad() and IsInKeyFrame() as the loop does at that point
template <class M, class KF, class MP, class DistOf>
int fuse(M& m, KF* kf, const std::vector<MP*>& vpMapPoints, float th, DistOf dist_of, float gx, float gy) {
  FramePack pk;
  pack_keyframe(*kf, pk, gx, gy);
  GeometryPack g(vpMapPoints, [&](MP* p) -> unsigned {
    return ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u) | (p->IsInKeyFrame(kf) ? ORBFE_MPF_SKIP : 0u);
  }, dist_of);
  const auto Tcw = kf->GetPose();
  const auto Ow = kf->GetCameraCenter();
  std::vector<int32_t> best;
  m.Fuse(pk.v, mat_floats(Tcw), mat_floats(Ow), g.view(), kf->mfLogScaleFactor, th, best);
  int nFused = 0;
  for (size_t i = 0; i < vpMapPoints.size(); i++) {
    MP* pMP = vpMapPoints[i];
    if (best[i] < 0 || !pMP || pMP->isBad() || pMP->IsInKeyFrame(kf)) continue;
    MP* pMPinKF = kf->GetMapPoint(best[i]);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations())
          pMP->Replace(pMPinKF);
        else
          pMPinKF->Replace(pMP);
      }
    } else {
      pMP->AddObservation(kf, best[i]);
      kf->AddMapPoint(pMP, best[i]);
    }
    nFused++;
  }
  return nFused;
}

// Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:993-1120)
template <class M, class KF, class MP, class DistOf>
int fuse_sim3(M& m, KF* kf, const float* scw, const std::vector<MP*>& vpPoints, float th,
              std::vector<MP*>& vpReplacePoint, DistOf dist_of, float gx, float gy) {
  FramePack pk;
  pack_keyframe(*kf, pk, gx, gy);
  const std::set<MP*> spAlreadyFound = kf->GetMapPoints();
  GeometryPack g(vpPoints, [&](MP* p) -> unsigned {
    return ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u) | (spAlreadyFound.count(p) ? ORBFE_MPF_SKIP : 0u);
  }, dist_of);
  std::vector<int32_t> best;
  const int nFused = m.FuseSim3(pk.v, scw, g.view(), kf->mfLogScaleFactor, th, best);
  for (size_t i = 0; i < vpPoints.size(); i++) {
    if (best[i] < 0) continue;
    MP* pMPinKF = kf->GetMapPoint(best[i]);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
    } else {
      vpPoints[i]->AddObservation(kf, best[i]);
      kf->AddMapPoint(vpPoints[i], best[i]);
    }
  }
  return nFused;
}

// SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (:1122-1346); t1w / t2w: the poses'
// rows 0..2, r12 / t12 continuous CV_32F
template <class M, class KF, class MP, class DistOf>
int search_by_sim3(M& m, KF* k1, KF* k2, std::vector<MP*>& vpMatches12, float s12, const float* r12,
                   const float* t12, float th, DistOf dist_of, float gx, float gy) {
  FramePack p1, p2;
  pack_keyframe(*k1, p1, gx, gy);
  pack_keyframe(*k2, p2, gx, gy);
  const std::vector<MP*> mps1 = k1->GetMapPointMatches(), mps2 = k2->GetMapPointMatches();
  std::vector<bool> matched1(mps1.size(), false), matched2(mps2.size(), false);  // :1150-1162
  for (size_t i = 0; i < mps1.size(); i++)
    if (MP* pMP = vpMatches12[i]) {
      matched1[i] = true;
      const int idx2 = pMP->GetIndexInKeyFrame(k2);
      if (idx2 >= 0 && idx2 < (int)mps2.size()) matched2[idx2] = true;
    }
  // SKIP = vbAlreadyMatched, by keypoint position (set after packing: flag_of sees the MapPoint only)
  auto present = [](MP* p) -> unsigned { return ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u); };
  GeometryPack g1(mps1, present, dist_of), g2(mps2, present, dist_of);
  for (size_t i = 0; i < mps1.size(); i++)
    if (mps1[i] && matched1[i]) g1.flags[i] |= ORBFE_MPF_SKIP;
  for (size_t i = 0; i < mps2.size(); i++)
    if (mps2[i] && matched2[i]) g2.flags[i] |= ORBFE_MPF_SKIP;
  const auto T1w = k1->GetPose(), T2w = k2->GetPose();
  std::vector<int32_t> m12;
  const int nFound = m.SearchBySim3(p1.v, p2.v, g1.view(), g2.view(), mat_floats(T1w), mat_floats(T2w), s12, r12,
                                    t12, k1->mfLogScaleFactor, k2->mfLogScaleFactor, th, m12);
  for (size_t i = 0; i < mps1.size(); i++)
    if (m12[i] >= 0) vpMatches12[i] = mps2[m12[i]];
  return nFound;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (:414-534); Pt has .x / .y
template <class M, class F, class Pt>
int search_for_initialization(M& m, F& f1, F& f2, std::vector<Pt>& vbPrevMatched, std::vector<int>& vnMatches12,
                              int window_size) {
  FramePack p1, p2;
  pack_frame(f1, f1.mvpMapPoints, p1);
  pack_frame(f2, f2.mvpMapPoints, p2);
  std::vector<float> prev(2 * vbPrevMatched.size());
  for (size_t i = 0; i < vbPrevMatched.size(); i++) {
    prev[2 * i] = vbPrevMatched[i].x;
    prev[2 * i + 1] = vbPrevMatched[i].y;
  }
  std::vector<int32_t> m12;
  const int n = m.SearchForInitialization(p1.v, p2.v, prev, m12, window_size);
  vnMatches12.assign(m12.begin(), m12.end());
  for (size_t i = 0; i < vbPrevMatched.size(); i++) {  // updated in place (:528-531)
    vbPrevMatched[i].x = prev[2 * i];
    vbPrevMatched[i].y = prev[2 * i + 1];
  }
  return n;
}

}  // namespace orbfe_adapter
#endif
