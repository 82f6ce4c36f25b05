// TEST-ONLY definitions of the cvstub MapPoint / KeyFrame methods (MapPoint.h, KeyFrame.h), written
// for the matcher adapter tests from the behaviour src/MapPoint.cc and src/KeyFrame.cc document:
// the same mutex per member, the same observation counting (a stereo observation counts twice,
// MapPoint.cc:128-139), the replaced point taking over the observations (:207-245), the normal /
// scale-invariance distances from the reference KeyFrame (:369-401) and the distinctive descriptor
// as the one with the least median distance to the others (:272-337). No Map, no covisibility.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {

namespace {
cv::Mat vec3(const float* v) {
  cv::Mat m(3, 1, CV_32F);
  std::memcpy(m.data, v, 3 * sizeof(float));
  return m;
}
int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}
}  // namespace

// ---- MapPoint -----------------------------------------------------------------------------------
MapPoint::MapPoint(const cv::Mat& Pos, KeyFrame* pRefKF, Map* pMap)
    : nObs(0), mTrackProjX(0), mTrackProjY(0), mTrackProjXR(0), mbTrackInView(false), mnTrackScaleLevel(0),
      mTrackViewCos(0), mpRefKF(pRefKF), mbBad(false), mpReplaced(nullptr), mfMinDistance(0), mfMaxDistance(0),
      mpMap(pMap) {
  mWorldPos = Pos.clone();
  mNormalVector = cv::Mat::zeros(3, 1, CV_32F);
  std::lock_guard<std::mutex> lock(mGlobalMutex);
  mnId = nNextId++;
}

void MapPoint::SetWorldPos(const cv::Mat& Pos) {
  std::lock_guard<std::mutex> l2(mGlobalMutex);
  std::lock_guard<std::mutex> lock(mMutexPos);
  mWorldPos = Pos.clone();
}
cv::Mat MapPoint::GetWorldPos() {
  std::lock_guard<std::mutex> lock(mMutexPos);
  return mWorldPos.clone();
}
cv::Mat MapPoint::GetNormal() {
  std::lock_guard<std::mutex> lock(mMutexPos);
  return mNormalVector.clone();
}
KeyFrame* MapPoint::GetReferenceKeyFrame() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mpRefKF;
}
std::map<KeyFrame*, size_t> MapPoint::GetObservations() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mObservations;
}
int MapPoint::Observations() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return nObs;
}
void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  if (mObservations.count(pKF)) return;
  mObservations[pKF] = idx;
  nObs += pKF->mvuRight[idx] >= 0 ? 2 : 1;
}
void MapPoint::EraseObservation(KeyFrame* pKF) {
  bool bad = false;
  {
    std::lock_guard<std::mutex> lock(mMutexFeatures);
    auto it = mObservations.find(pKF);
    if (it == mObservations.end()) return;
    nObs -= pKF->mvuRight[it->second] >= 0 ? 2 : 1;
    mObservations.erase(it);
    if (mpRefKF == pKF) mpRefKF = mObservations.empty() ? nullptr : mObservations.begin()->first;
    bad = nObs <= 2;
  }
  if (bad) SetBadFlag();
}
int MapPoint::GetIndexInKeyFrame(KeyFrame* pKF) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  auto it = mObservations.find(pKF);
  return it == mObservations.end() ? -1 : (int)it->second;
}
bool MapPoint::IsInKeyFrame(KeyFrame* pKF) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mObservations.count(pKF) > 0;
}
void MapPoint::SetBadFlag() {
  std::map<KeyFrame*, size_t> obs;
  {
    std::lock_guard<std::mutex> l1(mMutexFeatures);
    std::lock_guard<std::mutex> l2(mMutexPos);
    mbBad = true;
    obs.swap(mObservations);
  }
  for (auto& kv : obs) kv.first->EraseMapPointMatch(kv.second);
}
bool MapPoint::isBad() {
  std::lock_guard<std::mutex> l1(mMutexFeatures);
  std::lock_guard<std::mutex> l2(mMutexPos);
  return mbBad;
}
void MapPoint::Replace(MapPoint* pMP) {
  if (pMP->mnId == mnId) return;
  std::map<KeyFrame*, size_t> obs;
  {
    std::lock_guard<std::mutex> l1(mMutexFeatures);
    std::lock_guard<std::mutex> l2(mMutexPos);
    obs.swap(mObservations);
    mbBad = true;
    mpReplaced = pMP;
  }
  for (auto& kv : obs) {
    if (!pMP->IsInKeyFrame(kv.first)) {
      kv.first->ReplaceMapPointMatch(kv.second, pMP);
      pMP->AddObservation(kv.first, kv.second);
    } else {
      kv.first->EraseMapPointMatch(kv.second);
    }
  }
  pMP->ComputeDistinctiveDescriptors();
}
MapPoint* MapPoint::GetReplaced() {
  std::lock_guard<std::mutex> l1(mMutexFeatures);
  std::lock_guard<std::mutex> l2(mMutexPos);
  return mpReplaced;
}
void MapPoint::ComputeDistinctiveDescriptors() {
  std::vector<const uint8_t*> d;
  std::map<KeyFrame*, size_t> obs;
  {
    std::lock_guard<std::mutex> lock(mMutexFeatures);
    if (mbBad) return;
    obs = mObservations;
  }
  for (auto& kv : obs)
    if (!kv.first->isBad()) d.push_back(kv.first->mDescriptors.ptr<uint8_t>((int)kv.second));
  if (d.empty()) return;
  const size_t n = d.size();
  int best_median = 256;
  size_t best = 0;
  for (size_t i = 0; i < n; i++) {
    std::vector<int> di(n);
    for (size_t j = 0; j < n; j++) di[j] = hamming(d[i], d[j]);
    std::sort(di.begin(), di.end());
    const int median = di[(size_t)(0.5 * (n - 1))];
    if (median < best_median) {
      best_median = median;
      best = i;
    }
  }
  cv::Mat m(1, 32, CV_8U);
  std::memcpy(m.data, d[best], 32);
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  mDescriptor = m;
}
cv::Mat MapPoint::GetDescriptor() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mDescriptor.clone();
}
void MapPoint::UpdateNormalAndDepth() {
  std::map<KeyFrame*, size_t> obs;
  KeyFrame* ref;
  cv::Mat pos;
  {
    std::lock_guard<std::mutex> l1(mMutexFeatures);
    std::lock_guard<std::mutex> l2(mMutexPos);
    if (mbBad) return;
    obs = mObservations;
    ref = mpRefKF;
    pos = mWorldPos.clone();
  }
  if (obs.empty() || !ref) return;
  float normal[3] = {0.f, 0.f, 0.f};
  int n = 0;
  for (auto& kv : obs) {
    const cv::Mat o = kv.first->GetCameraCenter();
    float v[3];
    for (int k = 0; k < 3; k++) v[k] = pos.at<float>(k) - o.at<float>(k);
    const float len = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int k = 0; k < 3; k++) normal[k] += v[k] / len;
    n++;
  }
  const cv::Mat o = ref->GetCameraCenter();
  float pc[3];
  for (int k = 0; k < 3; k++) pc[k] = pos.at<float>(k) - o.at<float>(k);
  const float dist = std::sqrt(pc[0] * pc[0] + pc[1] * pc[1] + pc[2] * pc[2]);
  const int level = ref->mvKeysUn[obs[ref]].octave;
  const float level_scale = ref->mvScaleFactors[level];
  const int nlevels = ref->mnScaleLevels;
  for (int k = 0; k < 3; k++) normal[k] /= n;
  std::lock_guard<std::mutex> lock(mMutexPos);
  mfMaxDistance = dist * level_scale;
  mfMinDistance = mfMaxDistance / ref->mvScaleFactors[nlevels - 1];
  mNormalVector = vec3(normal);
}
float MapPoint::GetMinDistanceInvariance() {
  std::lock_guard<std::mutex> lock(mMutexPos);
  return 0.8f * mfMinDistance;
}
float MapPoint::GetMaxDistanceInvariance() {
  std::lock_guard<std::mutex> lock(mMutexPos);
  return 1.2f * mfMaxDistance;
}

// ---- KeyFrame -----------------------------------------------------------------------------------
KeyFrame::KeyFrame(Frame& F, Map*, KeyFrameDatabase*)
    : mfGridElementWidthInv(F.mfGridElementWidthInv), mfGridElementHeightInv(F.mfGridElementHeightInv),
      fx(F.fx), fy(F.fy), cx(F.cx), cy(F.cy), invfx(1.f / F.fx), invfy(1.f / F.fy), mbf(F.mbf), mb(F.mb), N(F.N),
      mvKeys(F.mvKeys), mvKeysUn(F.mvKeysUn), mvuRight(F.mvuRight), mvDepth(F.mvDepth),
      mDescriptors(F.mDescriptors.clone()), mFeatVec(F.mFeatVec), mnScaleLevels(F.mnScaleLevels),
      mfScaleFactor(F.mfScaleFactor), mfLogScaleFactor(F.mfLogScaleFactor), mvScaleFactors(F.mvScaleFactors),
      mvLevelSigma2(F.mvLevelSigma2), mvInvLevelSigma2(F.mvInvLevelSigma2), mnMinX((int)F.mnMinX),
      mnMinY((int)F.mnMinY), mnMaxX((int)F.mnMaxX), mnMaxY((int)F.mnMaxY), mvpMapPoints(F.mvpMapPoints),
      mbBad(false) {
  mnId = nNextId++;
  SetPose(F.mTcw);
}
void KeyFrame::SetPose(const cv::Mat& Tcw_) {
  std::lock_guard<std::mutex> lock(mMutexPose);
  Tcw = Tcw_.clone();
  // Ow = -Rcw^T tcw, Twc = [Rcw^T | Ow]
  Ow = cv::Mat(3, 1, CV_32F);
  Twc = cv::Mat::eye(4, 4, CV_32F);
  for (int i = 0; i < 3; i++) {
    float s = 0.f;
    for (int k = 0; k < 3; k++) {
      s -= Tcw.at<float>(k, i) * Tcw.at<float>(k, 3);
      Twc.at<float>(i, k) = Tcw.at<float>(k, i);
    }
    Ow.at<float>(i) = s;
    Twc.at<float>(i, 3) = s;
  }
}
cv::Mat KeyFrame::GetPose() {
  std::lock_guard<std::mutex> lock(mMutexPose);
  return Tcw.clone();
}
cv::Mat KeyFrame::GetPoseInverse() {
  std::lock_guard<std::mutex> lock(mMutexPose);
  return Twc.clone();
}
cv::Mat KeyFrame::GetCameraCenter() {
  std::lock_guard<std::mutex> lock(mMutexPose);
  return Ow.clone();
}
cv::Mat KeyFrame::GetRotation() {
  std::lock_guard<std::mutex> lock(mMutexPose);
  cv::Mat R(3, 3, CV_32F);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R.at<float>(i, j) = Tcw.at<float>(i, j);
  return R;
}
cv::Mat KeyFrame::GetTranslation() {
  std::lock_guard<std::mutex> lock(mMutexPose);
  cv::Mat t(3, 1, CV_32F);
  for (int i = 0; i < 3; i++) t.at<float>(i) = Tcw.at<float>(i, 3);
  return t;
}
void KeyFrame::AddMapPoint(MapPoint* pMP, const size_t& idx) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  mvpMapPoints[idx] = pMP;
}
void KeyFrame::EraseMapPointMatch(const size_t& idx) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  mvpMapPoints[idx] = nullptr;
}
void KeyFrame::ReplaceMapPointMatch(const size_t& idx, MapPoint* pMP) { mvpMapPoints[idx] = pMP; }
std::set<MapPoint*> KeyFrame::GetMapPoints() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  std::set<MapPoint*> s;
  for (MapPoint* p : mvpMapPoints)
    if (p && !p->isBad()) s.insert(p);
  return s;
}
std::vector<MapPoint*> KeyFrame::GetMapPointMatches() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mvpMapPoints;
}
MapPoint* KeyFrame::GetMapPoint(const size_t& idx) {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mvpMapPoints[idx];
}
void KeyFrame::SetBadFlag() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  mbBad = true;
}
bool KeyFrame::isBad() {
  std::lock_guard<std::mutex> lock(mMutexFeatures);
  return mbBad;
}

}  // namespace ORB_SLAM2
