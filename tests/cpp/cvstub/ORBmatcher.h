// TEST-ONLY declaration of the reference's public ORBmatcher interface (include/ORBmatcher.h:37-126)
// written over the cvstub types, so that adapter/ORBmatcher_gpu.cc -- which defines every one of
// these methods on liborbfe.so -- compiles and runs here (tests/cpp/matcher_e2e.cpp,
// matcher_tsan.cpp). tests/test_reference_pins.py checks every method's parameter list against
// the reference header when it is present.
#ifndef ORBFE_TEST_STUB_ORBMATCHER_H
#define ORBFE_TEST_STUB_ORBMATCHER_H

#include <set>
#include <vector>

#include <opencv2/core.hpp>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {

class ORBmatcher {
 public:
  ORBmatcher(float nnratio = 0.6, bool checkOri = true);

  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);

  int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3);

  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);

  int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                         const float th, const int ORBdist);

  int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                         std::vector<MapPoint*>& vpMatched, int th);

  int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
  int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);

  int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                              std::vector<int>& vnMatches12, int windowSize = 10);

  int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                             std::vector<pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo);

  int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                   const cv::Mat& R12, const cv::Mat& t12, const float th);

  int Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th = 3.0);

  int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
           vector<MapPoint*>& vpReplacePoint);

 public:
  static const int TH_LOW;
  static const int TH_HIGH;
  static const int HISTO_LENGTH;

 protected:
  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2

#endif
