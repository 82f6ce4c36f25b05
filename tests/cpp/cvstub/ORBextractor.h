// TEST-ONLY declaration of ORB_SLAM2::ORBextractor for compiling adapter/ORBextractor_gpu.cc
// here (tests/cpp/adapter_e2e.cpp). It declares the public interface and the data members of the
// reference's include/ORBextractor.h:47-126 that the adapter defines or fills, in the header's
// member order, over the cvstub types; the reference's private helper methods (ComputePyramid,
// ComputeKeyPointsOctTree, DistributeOctTree, ComputeKeyPointsOld), which the adapter does not
// define, are left out. tests/test_reference_pins.py checks the member names against the
// reference header when it is present.
#ifndef ORBFE_TEST_STUB_ORBEXTRACTOR_H
#define ORBFE_TEST_STUB_ORBEXTRACTOR_H

#include <vector>

#include <opencv2/core.hpp>

namespace ORB_SLAM2 {

class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
  ~ORBextractor() {}

  void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                  cv::OutputArray descriptors);

  int GetLevels() { return nlevels; }
  float GetScaleFactor() { return scaleFactor; }
  std::vector<float> GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  std::vector<cv::Mat> mvImagePyramid;

 protected:
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;

  std::vector<int> mnFeaturesPerLevel;
  std::vector<int> umax;

  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;
};

}  // namespace ORB_SLAM2

#endif
