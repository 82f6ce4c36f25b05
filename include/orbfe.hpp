/*
 * orbfe.hpp -- header-only C++17 facade over the liborbfe.so C ABI (include/orbfe.h).
 *
 * Mirrors the reference classes without OpenCV types so it builds anywhere:
 *   orbfe::Extractor  ~ ORB_SLAM2::ORBextractor  (include/ORBextractor.h:56-100)
 *   orbfe::Matcher    ~ ORB_SLAM2::ORBmatcher    (include/ORBmatcher.h:41-85)
 * The OpenCV-typed drop-in adapter a maintainer adds to the reference is built on this header
 * (INTEGRATION.md). Errors become orbfe::Error (the C ABI itself never throws).
 */
#ifndef ORBFE_HPP
#define ORBFE_HPP
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "orbfe.h"
#include "orbfe_keyframe.h"
#include "orbfe_stereo.h"

namespace orbfe {

struct Error : std::runtime_error {
  int status;
  Error(int st, const std::string& what)
      : std::runtime_error(what + " failed (" + std::to_string(st) + "): " + orbfe_last_error()),
        status(st) {}
};

inline int check(int st, const char* what) {
  if (st < 0) throw Error(st, what);
  return st;
}

using KeyPoint = orbfe_keypoint;  // cv::KeyPoint field order, 28 bytes

// A view of one pyramid level (ORBextractor::mvImagePyramid[l]); valid until the next call.
struct LevelView {
  const uint8_t* data = nullptr;
  int rows = 0, cols = 0;
  size_t step = 0;
};

class Extractor {
 public:
  // ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) (ORBextractor.h:56-57)
  Extractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
            int device = 0)
      : nlevels_(nlevels), scaleFactor_(scaleFactor) {
    check(orbfe_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device, &h_),
          "orbfe_extractor_create");
    scale_.resize(nlevels);
    inv_.resize(nlevels);
    s2_.resize(nlevels);
    is2_.resize(nlevels);
    fpl_.resize(nlevels);
    check(orbfe_get_scale_tables(h_, scale_.data(), inv_.data(), s2_.data(), is2_.data(), fpl_.data()),
          "orbfe_get_scale_tables");
  }
  ~Extractor() {
    if (h_) orbfe_extractor_destroy(h_);
  }
  Extractor(const Extractor&) = delete;
  Extractor& operator=(const Extractor&) = delete;
  Extractor(Extractor&& o) noexcept { *this = std::move(o); }
  Extractor& operator=(Extractor&& o) noexcept {
    std::swap(h_, o.h_);
    std::swap(nlevels_, o.nlevels_);
    std::swap(scaleFactor_, o.scaleFactor_);
    scale_.swap(o.scale_);
    inv_.swap(o.inv_);
    s2_.swap(o.s2_);
    is2_.swap(o.is2_);
    fpl_.swap(o.fpl_);
    return *this;
  }

  // operator()(image, mask, keypoints, descriptors) (ORBextractor.h:66-68): 8-bit grayscale
  // rows x cols with row step `step`; keypoints in level order, descriptors n x 32.
  void operator()(const uint8_t* image, int rows, int cols, size_t step, std::vector<KeyPoint>& keypoints,
                  std::vector<uint8_t>& descriptors) {
    keypoints.clear();
    descriptors.clear();
    if (rows <= 0 || cols <= 0) return;  // ORBextractor.cc:1044-1045
    const int cap = check(orbfe_max_keypoints(h_, rows, cols), "orbfe_max_keypoints");
    keypoints.resize(cap);
    descriptors.resize((size_t)cap * ORBFE_DESC_BYTES);
    int n = 0;
    check(orbfe_extract(h_, image, rows, cols, step, keypoints.data(), cap, descriptors.data(), &n),
          "orbfe_extract");
    keypoints.resize(n);
    descriptors.resize((size_t)n * ORBFE_DESC_BYTES);
  }

  // mvImagePyramid[level] of the last call (ORBextractor.h:100): a view of the handle's host copy
  // of that image's pyramid (one DMA on the first access to the image, none when prefetched);
  // every level's view stays valid until the next call.
  LevelView level(int level, int image = 0) {
    LevelView v;
    check(orbfe_get_level(h_, image, level, &v.data, &v.rows, &v.cols, &v.step), "orbfe_get_level");
    return v;
  }
  // Copy each call's pyramid to the host beside the extraction (orbfe_extractor_set_host_pyramid).
  void SetHostPyramid(bool on) { check(orbfe_extractor_set_host_pyramid(h_, on ? 1 : 0), "set_host_pyramid"); }
  // Replay the launch sequence as a hipGraph per argument set (default off; orbfe_extractor_set_graphs).
  void SetGraphs(bool on) { check(orbfe_extractor_set_graphs(h_, on ? 1 : 0), "set_graphs"); }

  // getters (ORBextractor.h:70-98)
  int GetLevels() const { return nlevels_; }
  float GetScaleFactor() const { return scaleFactor_; }
  const std::vector<float>& GetScaleFactors() const { return scale_; }
  const std::vector<float>& GetInverseScaleFactors() const { return inv_; }
  const std::vector<float>& GetScaleSigmaSquares() const { return s2_; }
  const std::vector<float>& GetInverseScaleSigmaSquares() const { return is2_; }
  const std::vector<int32_t>& FeaturesPerLevel() const { return fpl_; }

  orbfe_extractor* handle() const { return h_; }

 private:
  orbfe_extractor* h_ = nullptr;
  int nlevels_ = 0;
  float scaleFactor_ = 0.f;
  std::vector<float> scale_, inv_, s2_, is2_;
  std::vector<int32_t> fpl_;
};

class Matcher {
 public:
  static constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39

  // ORBmatcher(nnratio = 0.6, checkOri = true) (ORBmatcher.h:41)
  explicit Matcher(float nnratio = 0.6f, bool checkOri = true, int device = 0) {
    check(orbfe_matcher_create(nnratio, checkOri ? 1 : 0, device, &m_), "orbfe_matcher_create");
  }
  ~Matcher() {
    if (m_) orbfe_matcher_destroy(m_);
  }
  Matcher(const Matcher&) = delete;
  Matcher& operator=(const Matcher&) = delete;

  // static int DescriptorDistance(const cv::Mat&, const cv::Mat&) (ORBmatcher.h:44)
  static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbfe_descriptor_distance(a, b); }

  // SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.h:48): best_idx[i] is the
  // keypoint MapPoint i takes (-1 none); apply in ascending i. Returns nmatches.
  int SearchByProjection(const orbfe_frame_view& F, const orbfe_local_mappoints& mps, float th,
                         std::vector<int32_t>& best_idx) {
    best_idx.assign(mps.m > 0 ? mps.m : 0, -1);
    int nm = 0;
    check(orbfe_search_by_projection_local(m_, &F, &mps, th, best_idx.data(), &nm),
          "orbfe_search_by_projection_local");
    return nm;
  }

  // SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.h:52); best_idx codes as in
  // orbfe.h (k <= -2: assignment to keypoint -2-k made and undone by the rotation filter).
  int SearchByProjection(const orbfe_frame_view& current, const orbfe_lastframe_mappoints& last,
                         const float tcw_cur[12], float th, bool mono, std::vector<int32_t>& best_idx) {
    best_idx.assign(last.n > 0 ? last.n : 0, -1);
    int nm = 0;
    check(orbfe_search_by_projection_lastframe(m_, &current, &last, tcw_cur, th, mono ? 1 : 0,
                                               best_idx.data(), &nm),
          "orbfe_search_by_projection_lastframe");
    return nm;
  }

  // SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo) (ORBmatcher.h:84-85):
  // pairs (idx1, idx2) in ascending idx1, as the reference returns them (ORBmatcher.cc:828-836).
  int SearchForTriangulation(const orbfe_frame_view& kf1, const orbfe_frame_view& kf2,
                             const orbfe_feature_vector& fv1, const orbfe_feature_vector& fv2,
                             const float f12[9], float ex, float ey,
                             std::vector<std::pair<size_t, size_t>>& pairs, bool onlyStereo) {
    std::vector<int32_t> m12(kf1.n > 0 ? kf1.n : 1, -1);
    int nm = 0;
    check(orbfe_search_for_triangulation(m_, &kf1, &kf2, &fv1, &fv2, f12, ex, ey, onlyStereo ? 1 : 0,
                                         m12.data(), &nm),
          "orbfe_search_for_triangulation");
    pairs.clear();
    pairs.reserve(nm);
    for (int i = 0; i < kf1.n; i++)
      if (m12[i] >= 0) pairs.emplace_back((size_t)i, (size_t)m12[i]);
    return nm;
  }

  // ---- the remaining searches (orbfe_keyframe.h); outputs as documented there ----------------
  // SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.h:64): match_f[k] = KF keypoint or -1.
  int SearchByBoW(const orbfe_frame_view& kf, const orbfe_feature_vector& kf_fv, const orbfe_frame_view& F,
                  const orbfe_feature_vector& f_fv, std::vector<int32_t>& match_f) {
    match_f.assign(F.n > 0 ? F.n : 1, -1);
    int nm = 0;
    check(orbfe_search_by_bow_kf_frame(m_, &kf, &kf_fv, &F, &f_fv, match_f.data(), &nm), "SearchByBoW(KF, F)");
    match_f.resize(F.n > 0 ? F.n : 0);
    return nm;
  }
  // SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.h:65): match12[i] = KF2 keypoint or -1.
  int SearchByBoW12(const orbfe_frame_view& kf1, const orbfe_feature_vector& fv1, const orbfe_frame_view& kf2,
                    const orbfe_feature_vector& fv2, std::vector<int32_t>& match12) {
    match12.assign(kf1.n > 0 ? kf1.n : 1, -1);
    int nm = 0;
    check(orbfe_search_by_bow_kf_kf(m_, &kf1, &fv1, &kf2, &fv2, match12.data(), &nm), "SearchByBoW(KF, KF)");
    match12.resize(kf1.n > 0 ? kf1.n : 0);
    return nm;
  }
  // SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (ORBmatcher.h:56)
  int SearchByProjection(const orbfe_frame_view& current, const float tcw_cur[12],
                         const orbfe_mappoint_geometry& kf_points, const float* kf_angle, float log_scale_factor,
                         float th, int orb_dist, std::vector<int32_t>& best_idx) {
    best_idx.assign(kf_points.m > 0 ? kf_points.m : 1, -1);
    int nm = 0;
    check(orbfe_search_by_projection_keyframe(m_, &current, tcw_cur, &kf_points, kf_angle, log_scale_factor, th,
                                              orb_dist, best_idx.data(), &nm),
          "SearchByProjection(F, KF)");
    best_idx.resize(kf_points.m > 0 ? kf_points.m : 0);
    return nm;
  }
  // SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.h:60)
  int SearchByProjectionSim3(const orbfe_frame_view& kf, const float scw[12], const orbfe_mappoint_geometry& pts,
                             float log_scale_factor, int th, std::vector<int32_t>& best_idx) {
    best_idx.assign(pts.m > 0 ? pts.m : 1, -1);
    int nm = 0;
    check(orbfe_search_by_projection_sim3(m_, &kf, scw, &pts, log_scale_factor, th, best_idx.data(), &nm),
          "SearchByProjection(KF, Scw)");
    best_idx.resize(pts.m > 0 ? pts.m : 0);
    return nm;
  }
  // Fuse(pKF, vpMapPoints, th) (ORBmatcher.h:88): candidates; the caller applies and counts.
  int Fuse(const orbfe_frame_view& kf, const float tcw[12], const float ow[3], const orbfe_mappoint_geometry& pts,
           float log_scale_factor, float th, std::vector<int32_t>& best_idx) {
    best_idx.assign(pts.m > 0 ? pts.m : 1, -1);
    int n = 0;
    check(orbfe_fuse(m_, &kf, tcw, ow, &pts, log_scale_factor, th, best_idx.data(), &n), "Fuse(KF)");
    best_idx.resize(pts.m > 0 ? pts.m : 0);
    return n;
  }
  // Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (ORBmatcher.h:91)
  int FuseSim3(const orbfe_frame_view& kf, const float scw[12], const orbfe_mappoint_geometry& pts,
               float log_scale_factor, float th, std::vector<int32_t>& best_idx) {
    best_idx.assign(pts.m > 0 ? pts.m : 1, -1);
    int n = 0;
    check(orbfe_fuse_sim3(m_, &kf, scw, &pts, log_scale_factor, th, best_idx.data(), &n), "Fuse(KF, Scw)");
    best_idx.resize(pts.m > 0 ? pts.m : 0);
    return n;
  }
  // SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.h:69)
  int SearchBySim3(const orbfe_frame_view& kf1, const orbfe_frame_view& kf2, const orbfe_mappoint_geometry& mps1,
                   const orbfe_mappoint_geometry& mps2, const float t1w[12], const float t2w[12], float s12,
                   const float r12[9], const float t12[3], float lsf1, float lsf2, float th,
                   std::vector<int32_t>& match12) {
    match12.assign(kf1.n > 0 ? kf1.n : 1, -1);
    int n = 0;
    check(orbfe_search_by_sim3(m_, &kf1, &kf2, &mps1, &mps2, t1w, t2w, s12, r12, t12, lsf1, lsf2, th,
                               match12.data(), &n),
          "SearchBySim3");
    match12.resize(kf1.n > 0 ? kf1.n : 0);
    return n;
  }
  // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.h:77)
  int SearchForInitialization(const orbfe_frame_view& f1, const orbfe_frame_view& f2, std::vector<float>& prev_xy,
                              std::vector<int32_t>& match12, int window_size = 10) {
    match12.assign(f1.n > 0 ? f1.n : 1, -1);
    int nm = 0;
    check(orbfe_search_for_initialization(m_, &f1, &f2, prev_xy.data(), window_size, match12.data(), &nm),
          "SearchForInitialization");
    match12.resize(f1.n > 0 ? f1.n : 0);
    return nm;
  }
  // MapPoint::ComputeDistinctiveDescriptors for many MapPoints (MapPoint.cc:272-337)
  void ComputeDistinctiveDescriptors(const std::vector<int32_t>& offsets, const std::vector<uint8_t>& desc,
                                     std::vector<int32_t>& best_index) {
    const int n = offsets.empty() ? 0 : (int)offsets.size() - 1;
    best_index.assign(n, -1);
    check(orbfe_compute_distinctive_descriptors(m_, n, offsets.data(), desc.data(), best_index.data()),
          "ComputeDistinctiveDescriptors");
  }

  orbfe_matcher* handle() const { return m_; }

 private:
  orbfe_matcher* m_ = nullptr;
};

// Frame::ComputeStereoMatches (src/Frame.cc:522-700) with the reference's two extractors: the
// pyramids are those of the last call of `left` and `right` (image 0 of each). uRight / depth get
// one entry per left keypoint, -1 where unmatched (mvuRight / mvDepth). mb: see orbfe_stereo.h.
inline void ComputeStereoMatches(Extractor& left, Extractor& right, const std::vector<KeyPoint>& kl,
                                 const std::vector<uint8_t>& dl, const std::vector<KeyPoint>& kr,
                                 const std::vector<uint8_t>& dr, float mbf, float mb,
                                 std::vector<float>& uRight, std::vector<float>& depth) {
  uRight.assign(kl.size(), -1.0f);
  depth.assign(kl.size(), -1.0f);
  check(orbfe_compute_stereo_matches(left.handle(), 0, right.handle(), 0, kl.data(), dl.data(), (int)kl.size(),
                                     kr.data(), dr.data(), (int)kr.size(), mbf, mb, uRight.data(), depth.data()),
        "orbfe_compute_stereo_matches");
}

}  // namespace orbfe
#endif
