// ORBextractor_gpu.cc -- the drop-in replacement of the reference's src/ORBextractor.cc for a GPU
// build of lreithmayr/ORB_SLAM2_2021: every ORBextractor method the reference defines
// (include/ORBextractor.h:56-100) over liborbfe.so (include/orbfe.hpp). include/ORBextractor.h
// stays as it is, so Frame.cc / Tracking.cc compile and link unchanged; the GPU handle of each
// instance lives in a side table keyed by `this` (the header's inline destructor cannot free it:
// Tracking keeps its two or three extractors for the life of the process, Tracking.cc:125-131).
//
// Built only inside the reference's tree, where OpenCV and the reference headers exist
// (INTEGRATION.md section 4); anywhere else this translation unit is empty.
//
// ORBFE_ADAPTER_GPU_STEREO=1 (set when Frame_gpu.cc replaces Frame::ComputeStereoMatches): the
// public mvImagePyramid is left empty and no pyramid leaves the GPU. 0 (default): the CPU
// ComputeStereoMatches reads host copies of the levels.
#ifndef ORBFE_ADAPTER_GPU_STEREO
#define ORBFE_ADAPTER_GPU_STEREO 0
#endif
#if __has_include(<opencv2/core.hpp>) && __has_include("ORBextractor.h")

#include <cassert>
#include <cstddef>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>

#include <opencv2/core.hpp>

#include "ORBextractor.h"
#include "orbfe.hpp"

namespace ORB_SLAM2 {

namespace {
std::mutex g_mu;
std::map<const ORBextractor*, std::unique_ptr<orbfe::Extractor>>& handles() {
  static auto* m = new std::map<const ORBextractor*, std::unique_ptr<orbfe::Extractor>>();
  return *m;
}
orbfe::Extractor& gpu_of(const ORBextractor* e) {
  std::lock_guard<std::mutex> lk(g_mu);
  return *handles().at(e);
}
}  // namespace

// ORBextractor.cc:413-473: the scale / sigma tables and per-level budgets come from the library,
// computed with the reference's float arithmetic (tests/test_oracle_kat.py pins them)
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
  std::unique_ptr<orbfe::Extractor> g(
      new orbfe::Extractor(_nfeatures, _scaleFactor, _nlevels, _iniThFAST, _minThFAST));
  mvScaleFactor = g->GetScaleFactors();
  mvInvScaleFactor = g->GetInverseScaleFactors();
  mvLevelSigma2 = g->GetScaleSigmaSquares();
  mvInvLevelSigma2 = g->GetInverseScaleSigmaSquares();
  mnFeaturesPerLevel.assign(g->FeaturesPerLevel().begin(), g->FeaturesPerLevel().end());
  mvImagePyramid.resize(nlevels);
#if !ORBFE_ADAPTER_GPU_STEREO
  // the CPU Frame::ComputeStereoMatches reads mvImagePyramid after every call: the library copies
  // each pyramid down beside the rest of the extraction, so operator() pays no extra copy or wait
  g->SetHostPyramid(true);
#endif
  std::lock_guard<std::mutex> lk(g_mu);
  handles()[this] = std::move(g);
}

// ORBextractor.cc:1041-1103
void ORBextractor::operator()(cv::InputArray _image, cv::InputArray /*_mask: ignored, :65*/,
                              std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors) {
  if (_image.empty()) return;  // :1044-1045
  cv::Mat image = _image.getMat();
  assert(image.type() == CV_8UC1);  // :1048
  orbfe::Extractor& g = gpu_of(this);
  // cv::KeyPoint is orbfe_keypoint's layout (pt.x, pt.y, size, angle, response, octave, class_id):
  // the keypoints land in the caller's vector directly
  static_assert(sizeof(cv::KeyPoint) == sizeof(orbfe_keypoint), "cv::KeyPoint is 28 bytes");
  static_assert(offsetof(cv::KeyPoint, pt) == offsetof(orbfe_keypoint, x) &&
                    offsetof(cv::KeyPoint, pt) + sizeof(float) == offsetof(orbfe_keypoint, y) &&
                    sizeof(cv::KeyPoint::pt) == 2 * sizeof(float) &&
                    offsetof(cv::KeyPoint, size) == offsetof(orbfe_keypoint, size) &&
                    offsetof(cv::KeyPoint, angle) == offsetof(orbfe_keypoint, angle) &&
                    offsetof(cv::KeyPoint, response) == offsetof(orbfe_keypoint, response) &&
                    offsetof(cv::KeyPoint, octave) == offsetof(orbfe_keypoint, octave) &&
                    offsetof(cv::KeyPoint, class_id) == offsetof(orbfe_keypoint, class_id),
                "cv::KeyPoint's fields sit where orbfe_keypoint's do");
  const int cap = orbfe::check(orbfe_max_keypoints(g.handle(), image.rows, image.cols), "orbfe_max_keypoints");
  thread_local std::vector<uint8_t> desc;  // one operator() per thread at a time (Frame.cc:113-116)
  desc.resize((size_t)cap * 32);
  _keypoints.resize(cap);
  int n = 0;
  orbfe::check(orbfe_extract(g.handle(), image.data, image.rows, image.cols, image.step,
                             reinterpret_cast<orbfe_keypoint*>(_keypoints.data()), cap, desc.data(), &n),
               "orbfe_extract");
  _keypoints.resize(n);
  if (n == 0) {
    _descriptors.release();  // :1062-1063
  } else {
    _descriptors.create(n, 32, CV_8U);
    std::memcpy(_descriptors.getMat().data, desc.data(), (size_t)n * 32);
  }
#if !ORBFE_ADAPTER_GPU_STEREO
  // the public mvImagePyramid (ORBextractor.h:100): headers over the handle's host copy of this
  // call's pyramid (every level at once, prefetched during the extraction), valid until the next
  // call, as the reference's own levels are; Frame::ComputeStereoMatches reads them right after
  for (int l = 0; l < nlevels; l++) {
    const orbfe::LevelView v = g.level(l);
    mvImagePyramid[l] = cv::Mat(v.rows, v.cols, CV_8UC1, const_cast<uint8_t*>(v.data), v.step);
  }
#else
  // a build with Frame_gpu.cc reads the device pyramids (orbfe_compute_stereo_matches); nothing
  // else in the reference reads mvImagePyramid (Frame.cc:529,620-640 are its only readers), so
  // no level is copied to the host
#endif
}

}  // namespace ORB_SLAM2

// the GPU handle of an ORBextractor, for Frame_gpu.cc's ComputeStereoMatches
orbfe_extractor* orbfe_adapter_extractor_handle(const ORB_SLAM2::ORBextractor* e) {
  return ORB_SLAM2::gpu_of(e).handle();
}

#endif
