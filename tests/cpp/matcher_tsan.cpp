// adapter/ORBmatcher_gpu.cc's packers under ThreadSanitizer (CPU, no device): the keyframe searches
// that read MapPoint::mfMinDistance / mfMaxDistance -- relocalisation's SearchByProjection(F, pKF,
// sFound, th, ORBdist) on a Tracking thread, LoopClosing's SearchByProjection(pKF, Scw, ...),
// Fuse(pKF, Scw, ...) and SearchBySim3 on another, LocalMapping's Fuse(pKF, vpMapPoints) on a
// third -- while a LocalMapping-style writer runs MapPoint::UpdateNormalAndDepth and SetWorldPos
// on the same MapPoints (the writes MapPoint.cc:396-398 makes under mMutexPos). The adapter is
// built with a recording matcher (tsan_matcher.h) in place of the GPU.
//   matcher_tsan            the adapter as shipped: must run clean (exit 0)
//   matcher_tsan --control  adds a reader of the same members without the lock: ThreadSanitizer
//                           must report it (exit 66), which shows the clean run means something
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <set>
#include <thread>
#include <vector>

#include "ORBmatcher.h"

using namespace ORB_SLAM2;

extern "C" int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b) {  // DescriptorDistance's link
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

struct orbfe_test_access {
  static float unlocked_min(MapPoint* p) { return p->mfMinDistance; }  // the race the adapter must not have
};

namespace {
void fill_frame(Frame& F, int n, unsigned seed) {
  F.N = n;
  F.mvKeys.resize(n);
  for (int i = 0; i < n; i++) {
    const float x = 20.f + (float)((seed * 131u + i * 977u) % 1200u), y = 20.f + (float)((seed * 71u + i * 389u) % 330u);
    F.mvKeys[i] = cv::KeyPoint(x, y, 31.f, (float)(i % 360), 1.f, i % 8, -1);
  }
  F.mvKeysUn = F.mvKeys;
  F.mvuRight.assign(n, -1.f);
  F.mvDepth.assign(n, -1.f);
  F.mDescriptors = cv::Mat(n, 32, CV_8U);
  for (int i = 0; i < n * 32; i++) F.mDescriptors.data[i] = (uint8_t)(seed * 13u + i * 7u);
  F.mvpMapPoints.assign(n, nullptr);
  F.mvbOutlier.assign(n, false);
  F.mnScaleLevels = 8;
  F.mfScaleFactor = 1.2f;
  F.mfLogScaleFactor = 0.18232156f;
  F.mvScaleFactors = {1.f, 1.2f, 1.44f, 1.728f, 2.0736f, 2.48832f, 2.985984f, 3.5831808f};
  F.mvLevelSigma2 = {1.f, 1.44f, 2.0736f, 2.985984f, 4.2998f, 6.1917f, 8.9161f, 12.8392f};
  F.mvInvScaleFactors = F.mvScaleFactors;
  F.mvInvLevelSigma2 = F.mvLevelSigma2;
  F.mTcw = cv::Mat::eye(4, 4, CV_32F);
  F.mTcw.at<float>(2, 3) = -(float)seed;
  F.mFeatVec.addFeature(1, 0);
}
}  // namespace

int main(int argc, char** argv) {
  const bool control = argc > 1 && std::strcmp(argv[1], "--control") == 0;
  Frame::fx = Frame::fy = 718.856f;
  Frame::cx = 607.1928f;
  Frame::cy = 185.2157f;
  Frame::mnMaxX = 1241.f;
  Frame::mnMaxY = 376.f;
  Frame::mfGridElementWidthInv = 64.f / 1241.f;
  Frame::mfGridElementHeightInv = 48.f / 376.f;

  const int n = 160;
  Frame F0, F1, F2;
  fill_frame(F0, n, 0);
  fill_frame(F1, n, 1);
  fill_frame(F2, n, 2);
  KeyFrame K0(F0, nullptr, nullptr), K1(F1, nullptr, nullptr);
  std::vector<std::unique_ptr<MapPoint>> pool;
  for (int i = 0; i < n; i += 2) {
    cv::Mat X(3, 1, CV_32F);
    X.at<float>(0) = 0.01f * i;
    X.at<float>(1) = 0.5f;
    X.at<float>(2) = 5.f + 0.1f * i;
    pool.emplace_back(new MapPoint(X, &K0, nullptr));
    MapPoint* p = pool.back().get();
    p->AddObservation(&K0, i);
    K0.AddMapPoint(p, i);
    if (i % 4 == 0) {
      p->AddObservation(&K1, i);
      K1.AddMapPoint(p, i);
    }
    p->ComputeDistinctiveDescriptors();
    p->UpdateNormalAndDepth();
  }
  std::vector<MapPoint*> pts;
  for (auto& p : pool) pts.push_back(p.get());

  const int iters = 60;
  std::atomic<int> running{3};
  std::thread writer([&] {  // LocalMapping: UpdateNormalAndDepth / SetWorldPos on every MapPoint
    int round = 0;
    while (running.load() > 0 || round < 2) {
      for (MapPoint* p : pts) {
        cv::Mat X = p->GetWorldPos();
        X.at<float>(2) += (round % 2) ? 1e-3f : -1e-3f;
        p->SetWorldPos(X);
        p->UpdateNormalAndDepth();
      }
      round++;
    }
  });
  std::thread tracking([&] {  // Tracking::Relocalization's projection search (Tracking.cc:1480)
    for (int it = 0; it < iters; it++) {
      Frame C = F2;
      std::set<MapPoint*> found;
      ORBmatcher m(0.9, true);
      m.SearchByProjection(C, &K0, found, 10, 100);
    }
    running--;
  });
  std::thread loop([&] {  // LoopClosing::ComputeSim3 / SearchAndFuse (LoopClosing.cc:402, :619)
    for (int it = 0; it < iters; it++) {
      ORBmatcher m(0.75, true);
      std::vector<MapPoint*> matched(K1.N, nullptr), repl(pts.size(), nullptr), m12 = K1.GetMapPointMatches();
      const cv::Mat S = K1.GetPose();
      m.SearchByProjection(&K1, S, pts, matched, 10);
      m.Fuse(&K1, S, pts, 4, repl);
      cv::Mat R = cv::Mat::eye(3, 3, CV_32F), t = cv::Mat::zeros(3, 1, CV_32F);
      m.SearchBySim3(&K1, &K0, m12, 1.f, R, t, 7.5f);
    }
    running--;
  });
  std::thread mapping([&] {  // LocalMapping::SearchInNeighbors' Fuse (LocalMapping.cc:531)
    for (int it = 0; it < iters; it++) {
      ORBmatcher m;
      m.Fuse(&K1, pts, 3.f);
      if (control) {
        volatile float sink = 0.f;
        for (MapPoint* p : pts) sink = sink + orbfe_test_access::unlocked_min(p);
      }
    }
    running--;
  });
  tracking.join();
  loop.join();
  mapping.join();
  writer.join();
  std::printf("OK %zu MapPoints, %d rounds per reader%s\n", pts.size(), iters, control ? " (control)" : "");
  return 0;
}
