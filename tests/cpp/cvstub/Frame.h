// TEST-ONLY declaration of the part of ORB_SLAM2::Frame that adapter/Frame_gpu.cc touches (the
// reference's include/Frame.h: ExtractORB :86, ComputeStereoMatches :124, the extractors :137,
// mK :143, mbf :153, N :163, mvKeys / mvKeysRight :168, mvuRight / mvDepth :173-174, mDescriptors /
// mDescriptorsRight :181), over the cvstub types, for tests/cpp/adapter_e2e.cpp. ExtractORB is
// defined in that test the way src/Frame.cc:296-302 defines it.
#ifndef ORBFE_TEST_STUB_FRAME_H
#define ORBFE_TEST_STUB_FRAME_H

#include <vector>

#include <opencv2/core.hpp>

#include "ORBextractor.h"

namespace ORB_SLAM2 {

class Frame {
 public:
  void ExtractORB(int flag, const cv::Mat& im);
  void ComputeStereoMatches();

  ORBextractor *mpORBextractorLeft = nullptr, *mpORBextractorRight = nullptr;
  cv::Mat mK;
  float mbf = 0.f;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysRight;
  std::vector<float> mvuRight;
  std::vector<float> mvDepth;
  cv::Mat mDescriptors, mDescriptorsRight;
};

}  // namespace ORB_SLAM2

#endif
