/*
 * orbfe_pack.hpp -- the reference-side packers of the drop-in adapter (adapter/ORBmatcher_gpu.cc):
 * ORB-SLAM2's object graph (Frame / KeyFrame / MapPoint, DBoW2::FeatureVector) to the
 * struct-of-arrays views of include/orbfe.h, and the results back onto the objects.
 *
 * Header-only templates over the reference's member and method NAMES (include/Frame.h,
 * include/MapPoint.h, Thirdparty/DBoW2/DBoW2/FeatureVector.h), so they instantiate on the real
 * classes in the adapter and on Frame-shaped test structs in tests/cpp/adapter_pack_test.cpp. No
 * OpenCV include: a cv::Mat is only touched through its public `data` pointer (the reference's
 * descriptor rows, GetWorldPos() and mTcw are continuous CV_8U / CV_32F matrices).
 *
 * A packer owns the arrays its view points into; keep it alive for the call. Flags and states are
 * read the way the reference's own loops read them:
 *   FramePack        Frame::mvKeysUn, mvuRight, mDescriptors, the MapPoint state of every keypoint
 *                    (NULL / Observations() == 0 / Observations() > 0: ORBmatcher.cc:91-93,
 *                    :1421-1423), scale tables, bounds, grid, camera (Frame.h:130-215)
 *   LocalMapPack     SearchByProjection(F, vpMapPoints, th): mbTrackInView, isBad(), Observations()
 *                    (a MapPoint assigned in the loop blocks its keypoint only with observations),
 *                    mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos, GetDescriptor()
 *                    (ORBmatcher.cc:45-133)
 *   LastFramePack    SearchByProjection(CurrentFrame, LastFrame, th, bMono): mvpMapPoints[i] !=
 *                    NULL, mvbOutlier[i], Observations(), GetWorldPos(), GetDescriptor(),
 *                    mvKeys[i].octave, mvKeysUn[i].angle, LastFrame.mTcw rows 0..2
 *                    (ORBmatcher.cc:1348-1491)
 *   CsrFeatureVector DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>, ascending node
 *                    ids, features in insertion order) as CSR (TemplatedVocabulary.h:1161-1174)
 * and the result appliers:
 *   apply_local_matches      F.mvpMapPoints[best[i]] = vpMapPoints[i] in ascending i (:127)
 *   apply_lastframe_matches  every assignment (best >= 0, and best <= -2 = made, then undone by
 *                            the rotation filter) in ascending i, then NULL for each undone
 *                            keypoint (:1434-1488): a keypoint assigned twice and undone once ends
 *                            NULL, as in the reference
 */
#ifndef ORBFE_PACK_HPP
#define ORBFE_PACK_HPP

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/orbfe.h"
#include "../include/orbfe_keyframe.h"

namespace orbfe_adapter {

template <class M>
inline const uint8_t* mat_bytes(const M& m) {
  return reinterpret_cast<const uint8_t*>(m.data);
}
template <class M>
inline const float* mat_floats(const M& m) {
  return reinterpret_cast<const float*>(m.data);
}

// Frame / KeyFrame -> orbfe_frame_view. `mps` = F.mvpMapPoints or pKF->GetMapPointMatches().
struct FramePack {
  std::vector<orbfe_keypoint> keys;
  std::vector<uint8_t> mp_state;
  orbfe_frame_view v{};
};

// (the reference's MapPoint / KeyFrame accessors are non-const member functions: every pointer
// below is to a non-const object)
template <class MP>
inline uint8_t mp_state_of(MP* p) {
  if (!p) return ORBFE_MP_NONE;
  return p->Observations() > 0 ? ORBFE_MP_OBSERVED : ORBFE_MP_PRESENT;
}

template <class F, class MP>
inline void pack_frame(const F& f, const std::vector<MP*>& mps, FramePack& p) {
  const int n = f.N;
  p.keys.resize(n);
  for (int i = 0; i < n; i++) {
    const auto& k = f.mvKeysUn[i];
    p.keys[i] = orbfe_keypoint{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave, k.class_id};
  }
  p.mp_state.resize(n);
  for (int i = 0; i < n; i++) p.mp_state[i] = mp_state_of(mps[i]);
  p.v = orbfe_frame_view{};
  p.v.n = n;
  p.v.keys_un = p.keys.data();
  p.v.u_right = f.mvuRight.data();
  p.v.descriptors = mat_bytes(f.mDescriptors);  // N x 32 CV_8U, continuous
  p.v.mp_state = p.mp_state.data();
  p.v.nlevels = f.mnScaleLevels;
  p.v.scale_factors = f.mvScaleFactors.data();
  p.v.level_sigma2 = f.mvLevelSigma2.data();
  p.v.min_x = f.mnMinX;
  p.v.max_x = f.mnMaxX;
  p.v.min_y = f.mnMinY;
  p.v.max_y = f.mnMaxY;
  p.v.grid_inv_w = f.mfGridElementWidthInv;
  p.v.grid_inv_h = f.mfGridElementHeightInv;
  p.v.fx = f.fx;
  p.v.fy = f.fy;
  p.v.cx = f.cx;
  p.v.cy = f.cy;
  p.v.bf = f.mbf;
  p.v.b = f.mb;
}

// KeyFrame -> orbfe_frame_view (orbfe_keyframe.h conventions): GetMapPointMatches() with bad
// MapPoints marked ORBFE_MP_BAD, the KeyFrame's `const int` bounds, and the float grid origin of
// the Frame its mGrid came from (Frame::mnMinX / mnMinY, statics of the reference's Frame)
template <class KF>
inline void pack_keyframe(KF& kf, FramePack& p, float grid_min_x, float grid_min_y) {
  const auto mps = kf.GetMapPointMatches();
  pack_frame(kf, mps, p);
  for (int i = 0; i < kf.N; i++)
    if (mps[i] && mps[i]->isBad()) p.mp_state[i] = ORBFE_MP_BAD;
  p.v.grid_origin_set = 1;
  p.v.grid_min_x = grid_min_x;
  p.v.grid_min_y = grid_min_y;
}

// vector<MapPoint*> -> orbfe_mappoint_geometry. flag_of(p) gives the flags (ORBFE_MPF_PRESENT /
// _BAD / _SKIP as each search defines them, orbfe_keyframe.h); dist_of(p, min, max) reads
// mfMinDistance / mfMaxDistance, protected members of the reference's MapPoint (MapPoint.h:151-152)
// that only a friend reads -- the adapter passes a lambda from inside ORBmatcher, which
// MapPoint.h befriends
struct GeometryPack {
  std::vector<uint8_t> flags, desc;
  std::vector<float> pos, nrm, dmin, dmax;
  orbfe_mappoint_geometry v{};

  template <class MP, class FlagOf, class DistOf>
  GeometryPack(const std::vector<MP*>& mps, FlagOf flag_of, DistOf dist_of) {
    const size_t m = mps.size();
    flags.assign(m, 0);
    desc.assign(m * 32, 0);
    pos.assign(m * 3, 0.f);
    nrm.assign(m * 3, 0.f);
    dmin.assign(m, 0.f);
    dmax.assign(m, 0.f);
    for (size_t i = 0; i < m; i++) {
      MP* p = mps[i];
      flags[i] = p ? (uint8_t)flag_of(p) : (uint8_t)0;
      if (!p || (flags[i] & ORBFE_MPF_BAD)) continue;
      const auto w = p->GetWorldPos();
      std::memcpy(&pos[i * 3], mat_floats(w), 3 * sizeof(float));
      const auto n = p->GetNormal();
      std::memcpy(&nrm[i * 3], mat_floats(n), 3 * sizeof(float));
      dist_of(p, dmin[i], dmax[i]);
      const auto d = p->GetDescriptor();
      std::memcpy(&desc[i * 32], mat_bytes(d), 32);
    }
    v.m = (int32_t)m;
    v.flags = flags.data();
    v.world_pos = pos.data();
    v.normal = nrm.data();
    v.min_distance = dmin.data();
    v.max_distance = dmax.data();
    v.descriptors = desc.data();
  }
  const orbfe_mappoint_geometry& view() const { return v; }
};

// vector<MapPoint*> of Tracking::SearchLocalPoints (after isInFrustum) -> orbfe_local_mappoints
struct LocalMapPack {
  std::vector<uint8_t> flags, desc;
  std::vector<float> px, py, pxr, vcos;
  std::vector<int32_t> level;
  orbfe_local_mappoints v{};

  template <class MP>
  explicit LocalMapPack(const std::vector<MP*>& mps) {
    const size_t m = mps.size();
    flags.assign(m, 0);
    desc.assign(m * 32, 0);
    px.assign(m, 0.f);
    py.assign(m, 0.f);
    pxr.assign(m, 0.f);
    vcos.assign(m, 0.f);
    level.assign(m, 0);
    for (size_t i = 0; i < m; i++) {
      MP* p = mps[i];
      uint8_t fl = (p->mbTrackInView ? ORBFE_MPF_TRACK_IN_VIEW : 0u) | (p->isBad() ? ORBFE_MPF_BAD : 0u) |
                   (p->Observations() > 0 ? ORBFE_MPF_OBSERVED : 0u);
      flags[i] = fl;
      if (!(fl & ORBFE_MPF_TRACK_IN_VIEW) || (fl & ORBFE_MPF_BAD)) continue;  // skipped (:55-59)
      px[i] = p->mTrackProjX;
      py[i] = p->mTrackProjY;
      pxr[i] = p->mTrackProjXR;
      level[i] = p->mnTrackScaleLevel;
      vcos[i] = p->mTrackViewCos;
      const auto d = p->GetDescriptor();  // a copy under the MapPoint's mutex (MapPoint.cc:339-343)
      std::memcpy(&desc[i * 32], mat_bytes(d), 32);
    }
    v.m = (int32_t)m;
    v.flags = flags.data();
    v.proj_x = px.data();
    v.proj_y = py.data();
    v.proj_xr = pxr.data();
    v.level = level.data();
    v.view_cos = vcos.data();
    v.descriptors = desc.data();
  }
  const orbfe_local_mappoints& view() const { return v; }
};

// LastFrame -> orbfe_lastframe_mappoints
struct LastFramePack {
  std::vector<uint8_t> flags, desc;
  std::vector<float> pos, angle;
  std::vector<int32_t> octave;
  orbfe_lastframe_mappoints v{};

  template <class F>
  explicit LastFramePack(const F& last) {
    const int n = last.N;
    flags.assign(n, 0);
    desc.assign((size_t)n * 32, 0);
    pos.assign((size_t)n * 3, 0.f);
    angle.assign(n, 0.f);
    octave.assign(n, 0);
    for (int i = 0; i < n; i++) {
      auto* p = last.mvpMapPoints[i];
      octave[i] = last.mvKeys[i].octave;
      angle[i] = last.mvKeysUn[i].angle;
      if (!p) continue;
      uint8_t fl = ORBFE_MPF_PRESENT | (last.mvbOutlier[i] ? ORBFE_MPF_OUTLIER : 0u) |
                   (p->Observations() > 0 ? ORBFE_MPF_OBSERVED : 0u);
      flags[i] = fl;
      if (fl & ORBFE_MPF_OUTLIER) continue;  // never projected (:1377)
      const auto w = p->GetWorldPos();       // 3x1 CV_32F
      std::memcpy(&pos[(size_t)i * 3], mat_floats(w), 3 * sizeof(float));
      const auto d = p->GetDescriptor();
      std::memcpy(&desc[(size_t)i * 32], mat_bytes(d), 32);
    }
    v.n = n;
    v.flags = flags.data();
    v.world_pos = pos.data();
    v.descriptors = desc.data();
    v.octave = octave.data();
    v.angle = angle.data();
    std::memcpy(v.tcw_last, mat_floats(last.mTcw), 12 * sizeof(float));  // 4x4 CV_32F, rows 0..2
  }
  const orbfe_lastframe_mappoints& view() const { return v; }
};

// DBoW2::FeatureVector -> orbfe_feature_vector
struct CsrFeatureVector {
  std::vector<uint32_t> ids;
  std::vector<int32_t> offsets, indices;
  orbfe_feature_vector v{};

  template <class FV>
  explicit CsrFeatureVector(const FV& fv) {
    ids.reserve(fv.size());
    offsets.reserve(fv.size() + 1);
    offsets.push_back(0);
    for (const auto& kv : fv) {  // std::map: ascending NodeId
      ids.push_back((uint32_t)kv.first);
      for (auto idx : kv.second) indices.push_back((int32_t)idx);
      offsets.push_back((int32_t)indices.size());
    }
    v.n_nodes = (int32_t)ids.size();
    v.node_ids = ids.data();
    v.offsets = offsets.data();
    v.indices = indices.data();
  }
  const orbfe_feature_vector& view() const { return v; }
};

// SearchByProjection(F, vpMapPoints, th): F.mvpMapPoints[bestIdx] = pMP in ascending MapPoint order
template <class MP>
inline void apply_local_matches(const std::vector<int32_t>& best, std::vector<MP*>& frame_mps,
                                const std::vector<MP*>& vpMapPoints) {
  for (size_t i = 0; i < best.size(); i++)
    if (best[i] >= 0) frame_mps[best[i]] = vpMapPoints[i];
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) and (CurrentFrame, pKF, ...): all
// assignments in loop order, then the rotation filter's NULLs
template <class MP>
inline void apply_lastframe_matches(const std::vector<int32_t>& best, std::vector<MP*>& current_mps,
                                    const std::vector<MP*>& source_mps) {
  for (size_t i = 0; i < best.size(); i++)
    if (best[i] >= 0 || best[i] <= -2) current_mps[best[i] >= 0 ? best[i] : -2 - best[i]] = source_mps[i];
  for (size_t i = 0; i < best.size(); i++)
    if (best[i] <= -2) current_mps[-2 - best[i]] = nullptr;
}

}  // namespace orbfe_adapter
#endif
