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

  // mvImagePyramid[level] of the last call (ORBextractor.h:100), host copy on first access.
  LevelView level(int level, int image = 0) {
    LevelView v;
    check(orbfe_get_level(h_, image, level, &v.data, &v.rows, &v.cols, &v.step), "orbfe_get_level");
    return v;
  }

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
