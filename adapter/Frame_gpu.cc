// Frame_gpu.cc -- Frame::ComputeStereoMatches (src/Frame.cc:522-700) of a GPU build of
// lreithmayr/ORB_SLAM2_2021, over the pyramids the two extractors left on the GPU in the
// ExtractORB calls just before (Frame.cc:113-116; adapter/ORBextractor_gpu.cc). The maintainer
// removes the method's body from src/Frame.cc and compiles this file beside it.
//
// Built only inside the reference's tree; anywhere else this
// translation unit is empty.
#if __has_include(<opencv2/core.hpp>) && __has_include("Frame.h")

#include <opencv2/core.hpp>

#include "Frame.h"
#include "ORBextractor.h"
#include "orbfe.hpp"

orbfe_extractor* orbfe_adapter_extractor_handle(const ORB_SLAM2::ORBextractor* e);  // ORBextractor_gpu.cc

namespace ORB_SLAM2 {

void Frame::ComputeStereoMatches() {
  mvuRight = std::vector<float>(N, -1.0f);  // :524-525
  mvDepth = std::vector<float>(N, -1.0f);
  if (N == 0) return;
  // the reference reads mb here before the constructor assigns it (:552 vs :149); the GPU call
  // takes it explicitly: the value the constructor is about to assign
  const float mbUsed = mbf / mK.at<float>(0, 0);
  const int st = orbfe_compute_stereo_matches(
      orbfe_adapter_extractor_handle(mpORBextractorLeft), 0, orbfe_adapter_extractor_handle(mpORBextractorRight), 0,
      reinterpret_cast<const orbfe_keypoint*>(mvKeys.data()), mDescriptors.ptr<uint8_t>(), N,  // 28-byte cv::KeyPoint
      reinterpret_cast<const orbfe_keypoint*>(mvKeysRight.data()),
      mDescriptorsRight.empty() ? nullptr : mDescriptorsRight.ptr<uint8_t>(), (int)mvKeysRight.size(), mbf, mbUsed,
      mvuRight.data(), mvDepth.data());
  if (st != ORBFE_OK) throw orbfe::Error(st, "orbfe_compute_stereo_matches");
}

}  // namespace ORB_SLAM2

#endif
