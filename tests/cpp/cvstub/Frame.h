// TEST-ONLY declaration of the part of ORB_SLAM2::Frame that the adapters touch, over the cvstub
// types, with the reference's member names (include/Frame.h):
//   adapter/Frame_gpu.cc (tests/cpp/adapter_e2e.cpp): ExtractORB :86, ComputeStereoMatches :124,
//     the extractors :137, mK :143, mbf :153, N :163, mvKeys / mvKeysRight :168, mvuRight /
//     mvDepth :173-174, mDescriptors / mDescriptorsRight :181;
//   adapter/ORBmatcher_gpu.cc (tests/cpp/matcher_e2e.cpp, matcher_tsan.cpp): the camera statics
//     fx..cy :144-147, mb :156, mvKeysUn :169, mFeatVec :178, mvpMapPoints :184, mvbOutlier :187,
//     the grid statics :190-191, mTcw :195, the scale members :207-212, the image-bound statics
//     :216-219.
// ExtractORB is defined by adapter_e2e.cpp the way src/Frame.cc:296-302 defines it.
// tests/test_reference_pins.py checks these names against the reference header when present.
#ifndef ORBFE_TEST_STUB_FRAME_H
#define ORBFE_TEST_STUB_FRAME_H

#include <vector>

#include <opencv2/core.hpp>

#include "DBoW2/FeatureVector.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {

class MapPoint;

class Frame {
 public:
  void ExtractORB(int flag, const cv::Mat& im);
  void ComputeStereoMatches();

  ORBextractor *mpORBextractorLeft = nullptr, *mpORBextractorRight = nullptr;
  cv::Mat mK;
  inline static float fx = 0.f;
  inline static float fy = 0.f;
  inline static float cx = 0.f;
  inline static float cy = 0.f;
  float mbf = 0.f;
  float mb = 0.f;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysRight;
  std::vector<cv::KeyPoint> mvKeysUn;
  std::vector<float> mvuRight;
  std::vector<float> mvDepth;
  DBoW2::FeatureVector mFeatVec;
  cv::Mat mDescriptors, mDescriptorsRight;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
  inline static float mfGridElementWidthInv = 0.f;
  inline static float mfGridElementHeightInv = 0.f;
  cv::Mat mTcw;
  int mnScaleLevels = 0;
  float mfScaleFactor = 0.f;
  float mfLogScaleFactor = 0.f;
  std::vector<float> mvScaleFactors;
  std::vector<float> mvInvScaleFactors;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;
  inline static float mnMinX = 0.f;
  inline static float mnMaxX = 0.f;
  inline static float mnMinY = 0.f;
  inline static float mnMaxY = 0.f;
};

}  // namespace ORB_SLAM2

#endif
