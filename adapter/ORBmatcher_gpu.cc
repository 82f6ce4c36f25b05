// ORBmatcher_gpu.cc -- the drop-in replacement of the reference's src/ORBmatcher.cc for a GPU
// build of lreithmayr/ORB_SLAM2_2021: every public ORBmatcher method (include/ORBmatcher.h:41-100)
// over liborbfe.so. The bodies are the templates of adapter/orbfe_adapter.hpp (pack the object
// graph, search on the GPU, apply in the reference's loop order), instantiated here on the real
// Frame / KeyFrame / MapPoint; tests/cpp/adapter_pack_test.cpp runs the same templates on
// Frame-shaped test structs.
//
// One line changes in the reference's include/MapPoint.h: `friend class ORBmatcher;` beside the
// protected mfMinDistance / mfMaxDistance (MapPoint.h:151-152), which the keyframe searches pass
// to the GPU as they are (MapPoint exposes only 0.8f / 1.2f times them). They are read under the
// MapPoint's mMutexPos, the mutex UpdateNormalAndDepth writes them under (MapPoint.cc:396-398) on
// the LocalMapping thread while Tracking / LoopClosing run these searches. The protected helpers
// CheckDistEpipolarLine, RadiusByViewingCos and ComputeThreeMaxima have no caller left outside
// the searches and are not defined.
//
// Built only inside the reference's tree; anywhere else this
// translation unit is empty.
#if __has_include(<opencv2/core.hpp>) && __has_include("ORBmatcher.h")

#include <map>
#include <memory>
#include <mutex>
#include <utility>

#include <opencv2/core.hpp>

#include "ORBmatcher.h"
#include "orbfe.hpp"
#include "orbfe_adapter.hpp"

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;  // ORBmatcher.cc:37-39
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

// The matcher behind the methods: liborbfe's facade. tests/cpp/matcher_tsan.cpp builds this file
// with a recording matcher in its place (no GPU) to run the packers under ThreadSanitizer.
#ifndef ORBFE_ADAPTER_MATCHER
#define ORBFE_ADAPTER_MATCHER orbfe::Matcher
#endif

namespace {
// one GPU matcher per (thread, nnratio, checkOri): the reference constructs ORBmatchers on the stack
// per call (Tracking.cc:889,1207, LocalMapping.cc:219), and the handles are thread-compatible only
ORBFE_ADAPTER_MATCHER& gpu_matcher(float nnratio, bool checkOri) {
  thread_local std::map<std::pair<float, bool>, std::unique_ptr<ORBFE_ADAPTER_MATCHER>> pool;
  std::unique_ptr<ORBFE_ADAPTER_MATCHER>& m = pool[{nnratio, checkOri}];
  if (!m) m.reset(new ORBFE_ADAPTER_MATCHER(nnratio, checkOri));
  return *m;
}
cv::Mat continuous(const cv::Mat& m) { return m.isContinuous() ? m : m.clone(); }
}  // namespace

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

// :1672-1688
int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orbfe_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  return orbfe_adapter::search_by_projection_local(gpu_matcher(mfNNratio, mbCheckOrientation), F, vpMapPoints, th);
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
  CurrentFrame.mTcw = continuous(CurrentFrame.mTcw);
  return orbfe_adapter::search_by_projection_lastframe(gpu_matcher(mfNNratio, mbCheckOrientation), CurrentFrame,
                                                       LastFrame, th, bMono);
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
  CurrentFrame.mTcw = continuous(CurrentFrame.mTcw);
  return orbfe_adapter::search_by_projection_keyframe(
      gpu_matcher(mfNNratio, mbCheckOrientation), CurrentFrame, pKF, sAlreadyFound, th, ORBdist,
      [](MapPoint* p, float& dmin, float& dmax) {  // under mMutexPos, as MapPoint.cc:403-447 reads them
        std::unique_lock<std::mutex> lock(p->mMutexPos);
        dmin = p->mfMinDistance;
        dmax = p->mfMaxDistance;
      });
}

int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                                   std::vector<MapPoint*>& vpMatched, int th) {
  const cv::Mat S = continuous(Scw);
  return orbfe_adapter::search_by_projection_sim3(
      gpu_matcher(mfNNratio, mbCheckOrientation), pKF, S.ptr<float>(), vpPoints, vpMatched, th,
      [](MapPoint* p, float& dmin, float& dmax) {  // under mMutexPos, as MapPoint.cc:403-447 reads them
        std::unique_lock<std::mutex> lock(p->mMutexPos);
        dmin = p->mfMinDistance;
        dmax = p->mfMaxDistance;
      },
      Frame::mnMinX, Frame::mnMinY);
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  return orbfe_adapter::search_by_bow(gpu_matcher(mfNNratio, mbCheckOrientation), pKF, F, vpMapPointMatches,
                                      Frame::mnMinX, Frame::mnMinY);
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
  return orbfe_adapter::search_by_bow12(gpu_matcher(mfNNratio, mbCheckOrientation), pKF1, pKF2, vpMatches12,
                                        Frame::mnMinX, Frame::mnMinY);
}

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
  return orbfe_adapter::search_for_initialization(gpu_matcher(mfNNratio, mbCheckOrientation), F1, F2, vbPrevMatched,
                                                  vnMatches12, windowSize);
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo) {
  // the epipole of KF1 in KF2 with the reference's own expression (:678-684)
  cv::Mat Cw = pKF1->GetCameraCenter();
  cv::Mat R2w = pKF2->GetRotation();
  cv::Mat t2w = pKF2->GetTranslation();
  cv::Mat C2 = R2w * Cw + t2w;
  const float invz = 1.0f / C2.at<float>(2);
  const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
  const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
  const cv::Mat F = continuous(F12);
  return orbfe_adapter::search_for_triangulation(gpu_matcher(mfNNratio, mbCheckOrientation), pKF1, pKF2,
                                                 F.ptr<float>(), ex, ey, vMatchedPairs, bOnlyStereo);
}

int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                             const cv::Mat& R12, const cv::Mat& t12, const float th) {
  const cv::Mat R = continuous(R12), t = continuous(t12);
  return orbfe_adapter::search_by_sim3(
      gpu_matcher(mfNNratio, mbCheckOrientation), pKF1, pKF2, vpMatches12, s12, R.ptr<float>(), t.ptr<float>(), th,
      [](MapPoint* p, float& dmin, float& dmax) {  // under mMutexPos, as MapPoint.cc:403-447 reads them
        std::unique_lock<std::mutex> lock(p->mMutexPos);
        dmin = p->mfMinDistance;
        dmax = p->mfMaxDistance;
      },
      Frame::mnMinX, Frame::mnMinY);
}

int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  return orbfe_adapter::fuse(
      gpu_matcher(mfNNratio, mbCheckOrientation), pKF, vpMapPoints, th,
      [](MapPoint* p, float& dmin, float& dmax) {  // under mMutexPos, as MapPoint.cc:403-447 reads them
        std::unique_lock<std::mutex> lock(p->mMutexPos);
        dmin = p->mfMinDistance;
        dmax = p->mfMaxDistance;
      },
      Frame::mnMinX, Frame::mnMinY);
}

int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
                     std::vector<MapPoint*>& vpReplacePoint) {
  const cv::Mat S = continuous(Scw);
  return orbfe_adapter::fuse_sim3(
      gpu_matcher(mfNNratio, mbCheckOrientation), pKF, S.ptr<float>(), vpPoints, th, vpReplacePoint,
      [](MapPoint* p, float& dmin, float& dmax) {  // under mMutexPos, as MapPoint.cc:403-447 reads them
        std::unique_lock<std::mutex> lock(p->mMutexPos);
        dmin = p->mfMinDistance;
        dmax = p->mfMaxDistance;
      },
      Frame::mnMinX, Frame::mnMinY);
}

}  // namespace ORB_SLAM2

#endif
