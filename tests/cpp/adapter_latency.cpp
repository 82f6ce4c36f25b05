// Latency of the drop-in adapters as the reference calls them (no checker linked: bench.py runs
// this for its c2_latency leg; tests/cpp/adapter_e2e.cpp is the parity test of the same code).
// adapter/ORBextractor_gpu.cc's operator() on one 1241x376 image (Frame::ExtractORB ->
// ORBextractor::operator(), ORBextractor.cc:1041-1103, with the cv::Mat outputs and the public
// mvImagePyramid), and the stereo Frame constructor's sequence (Frame.cc:113-125: two std::threads
// extracting, then adapter/Frame_gpu.cc's ComputeStereoMatches). Built twice (tests/cpp/Makefile):
// host pyramid (default) and ORBFE_ADAPTER_GPU_STEREO=1. Prints one "ADAPTER {json}" line.
// Exit: 0 ok, 77 no GPU.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include "Frame.h"
#include "ORBextractor.h"
#include "orbfe.hpp"
#include "orbfe_synth.h"

#ifndef ORBFE_ADAPTER_GPU_STEREO
#define ORBFE_ADAPTER_GPU_STEREO 0
#endif

namespace ORB_SLAM2 {
void Frame::ExtractORB(int flag, const cv::Mat& im) {  // src/Frame.cc:296-302
  if (flag == 0)
    (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors);
  else
    (*mpORBextractorRight)(im, cv::Mat(), mvKeysRight, mDescriptorsRight);
}
}  // namespace ORB_SLAM2

using ORB_SLAM2::Frame;
using ORB_SLAM2::ORBextractor;

static double p50(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
}
static double ms(const std::function<void()>& f) {
  const auto t0 = std::chrono::steady_clock::now();
  f();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const int rows = 376, cols = 1241;
  std::unique_ptr<ORBextractor> el, er;
  try {
    el.reset(new ORBextractor(2000, 1.2f, 8, 20, 7));
    er.reset(new ORBextractor(2000, 1.2f, 8, 20, 7));
  } catch (const orbfe::Error& e) {
    std::printf("no device: %s\n", e.what());
    return 77;
  }
  std::vector<uint8_t> left((size_t)rows * cols), right((size_t)rows * cols);
  if (orbfe_synth_frame(5, rows, cols, 0, left.data(), right.data(), cols) != 0) return 1;
  const cv::Mat L(rows, cols, CV_8UC1, left.data(), cols), R(rows, cols, CV_8UC1, right.data(), cols);
  Frame F;
  F.mpORBextractorLeft = el.get();
  F.mpORBextractorRight = er.get();
  F.mK = cv::Mat(3, 3, CV_32F);
  std::memset(F.mK.data, 0, 9 * sizeof(float));
  F.mK.at<float>(0, 0) = 718.856f;
  F.mK.at<float>(1, 1) = 718.856f;
  F.mK.at<float>(0, 2) = 607.1928f;
  F.mK.at<float>(1, 2) = 185.2157f;
  F.mK.at<float>(2, 2) = 1.f;
  F.mbf = 386.1448f;
  std::vector<cv::KeyPoint> kps;
  cv::Mat desc;
  std::vector<double> t_op, t_frame;
  for (int i = 0; i < iters + 10; i++) {
    const double a = ms([&] { (*el)(L, cv::Mat(), kps, desc); });
    const double b = ms([&] {
      std::thread tl(&Frame::ExtractORB, &F, 0, std::cref(L));
      std::thread tr(&Frame::ExtractORB, &F, 1, std::cref(R));
      tl.join();
      tr.join();
      F.N = (int)F.mvKeys.size();
      F.ComputeStereoMatches();
    });
    if (i >= 10) {
      t_op.push_back(a);
      t_frame.push_back(b);
    }
  }
  int matched = 0;
  for (float u : F.mvuRight) matched += u >= 0;
  std::printf("ADAPTER {\"gpu_stereo_build\": %d, \"operator_p50_ms\": %.4f, \"operator_p99_ms\": %.4f, "
              "\"stereo_frame_p50_ms\": %.4f, \"stereo_frame_p99_ms\": %.4f, \"iters\": %d, \"keypoints\": %zu, "
              "\"stereo_matched\": %d}\n",
              ORBFE_ADAPTER_GPU_STEREO, p50(t_op), pct(t_op, 0.99), p50(t_frame), pct(t_frame, 0.99), iters,
              kps.size(), matched);
  return 0;
}
