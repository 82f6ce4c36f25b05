// TEST-ONLY declaration of ORB_SLAM2::MapPoint over the cvstub types: the public interface and the
// members adapter/ORBmatcher_gpu.cc reads (the reference's include/MapPoint.h:40-158, same names
// and locking discipline: position, normal and the scale-invariance distances under mMutexPos,
// observations, descriptor and the bad flag under mMutexFeatures). The methods are defined in
// map_stub.cc with the behaviour src/MapPoint.cc documents; serialization, the Map and the
// tracking counters the searches never read are left out. Two test-only additions, marked below:
// friend access for the checker (tests/cpp/matcher_e2e.cpp reads mfMinDistance / mfMaxDistance
// the way the reference's ORBmatcher does) and nothing else. tests/test_reference_pins.py checks
// the member names against the reference header when present.
#ifndef ORBFE_TEST_STUB_MAPPOINT_H
#define ORBFE_TEST_STUB_MAPPOINT_H

#include <map>
#include <mutex>

#include <opencv2/core.hpp>

#include "Frame.h"

struct orbfe_test_access;  // TEST-ONLY: the checker's reader of the protected distances

namespace ORB_SLAM2 {

class KeyFrame;
class Map;
class Frame;

class MapPoint {
 public:
  MapPoint(const cv::Mat& Pos, KeyFrame* pRefKF, Map* pMap);

  void SetWorldPos(const cv::Mat& Pos);
  cv::Mat GetWorldPos();

  cv::Mat GetNormal();
  KeyFrame* GetReferenceKeyFrame();

  std::map<KeyFrame*, size_t> GetObservations();
  int Observations();

  void AddObservation(KeyFrame* pKF, size_t idx);
  void EraseObservation(KeyFrame* pKF);

  int GetIndexInKeyFrame(KeyFrame* pKF);
  bool IsInKeyFrame(KeyFrame* pKF);

  void SetBadFlag();
  bool isBad();

  void Replace(MapPoint* pMP);
  MapPoint* GetReplaced();

  void ComputeDistinctiveDescriptors();

  cv::Mat GetDescriptor();

  void UpdateNormalAndDepth();

  float GetMinDistanceInvariance();
  float GetMaxDistanceInvariance();

 public:
  long unsigned int mnId;
  inline static long unsigned int nNextId = 0;
  int nObs;

  // Variables used by the tracking
  float mTrackProjX;
  float mTrackProjY;
  float mTrackProjXR;
  bool mbTrackInView;
  int mnTrackScaleLevel;
  float mTrackViewCos;

  inline static std::mutex mGlobalMutex;

 protected:
  cv::Mat mWorldPos;
  std::map<KeyFrame*, size_t> mObservations;
  cv::Mat mNormalVector;
  cv::Mat mDescriptor;
  KeyFrame* mpRefKF;
  bool mbBad;
  MapPoint* mpReplaced;
  float mfMinDistance;
  float mfMaxDistance;
  Map* mpMap;
  std::mutex mMutexPos;
  std::mutex mMutexFeatures;

  // The reference's include/MapPoint.h gains this one line in the GPU build (INTEGRATION.md
  // section 3c): the adapter packs mfMinDistance / mfMaxDistance under mMutexPos
  friend class ORBmatcher;
  friend struct ::orbfe_test_access;  // TEST-ONLY
};

}  // namespace ORB_SLAM2

#endif
