// TEST-ONLY declaration of ORB_SLAM2::KeyFrame over the cvstub types: the constructor from a Frame,
// the pose and MapPoint accessors and the public const members adapter/ORBmatcher_gpu.cc reads
// (the reference's include/KeyFrame.h:44-245, same names; pose under mMutexPose, MapPoint slots
// under mMutexFeatures). Methods are defined in map_stub.cc with the behaviour src/KeyFrame.cc
// documents; the covisibility graph, spanning tree, BoW database, grid and serialization are left
// out. tests/test_reference_pins.py checks the member names against the reference header.
#ifndef ORBFE_TEST_STUB_KEYFRAME_H
#define ORBFE_TEST_STUB_KEYFRAME_H

#include <mutex>
#include <set>
#include <vector>

#include <opencv2/core.hpp>

#include "DBoW2/FeatureVector.h"
#include "Frame.h"

namespace ORB_SLAM2 {

class Map;
class MapPoint;
class Frame;
class KeyFrameDatabase;

class KeyFrame {
 public:
  KeyFrame(Frame& F, Map* pMap, KeyFrameDatabase* pKFDB);

  // Pose functions
  void SetPose(const cv::Mat& Tcw);
  cv::Mat GetPose();
  cv::Mat GetPoseInverse();
  cv::Mat GetCameraCenter();
  cv::Mat GetRotation();
  cv::Mat GetTranslation();

  // MapPoint observation functions
  void AddMapPoint(MapPoint* pMP, const size_t& idx);
  void EraseMapPointMatch(const size_t& idx);
  void ReplaceMapPointMatch(const size_t& idx, MapPoint* pMP);
  std::set<MapPoint*> GetMapPoints();
  std::vector<MapPoint*> GetMapPointMatches();
  MapPoint* GetMapPoint(const size_t& idx);

  void SetBadFlag();
  bool isBad();

 public:
  inline static long unsigned int nNextId = 0;
  long unsigned int mnId;

  // Grid (to speed up feature matching)
  const float mfGridElementWidthInv;
  const float mfGridElementHeightInv;

  // Calibration parameters
  const float fx, fy, cx, cy, invfx, invfy, mbf, mb;

  // Number of KeyPoints
  const int N;

  // KeyPoints, stereo coordinate and descriptors (all associated by an index)
  const std::vector<cv::KeyPoint> mvKeys;
  const std::vector<cv::KeyPoint> mvKeysUn;
  const std::vector<float> mvuRight;
  const std::vector<float> mvDepth;
  const cv::Mat mDescriptors;

  // BoW
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;

  // Scale
  const int mnScaleLevels;
  const float mfScaleFactor;
  const float mfLogScaleFactor;
  const std::vector<float> mvScaleFactors;
  const std::vector<float> mvLevelSigma2;
  const std::vector<float> mvInvLevelSigma2;

  // Image bounds and calibration
  const int mnMinX;
  const int mnMinY;
  const int mnMaxX;
  const int mnMaxY;

 protected:
  // SE3 Pose and camera center
  cv::Mat Tcw;
  cv::Mat Twc;
  cv::Mat Ow;

  // MapPoints associated to keypoints
  std::vector<MapPoint*> mvpMapPoints;

  bool mbBad;

  std::mutex mMutexPose;
  std::mutex mMutexFeatures;
};

}  // namespace ORB_SLAM2

#endif
