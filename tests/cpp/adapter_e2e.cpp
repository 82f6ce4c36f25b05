// The reference-side drop-in adapters (adapter/ORBextractor_gpu.cc, adapter/Frame_gpu.cc) compiled
// against test-only OpenCV / reference declarations (tests/cpp/cvstub/) and run the way the
// reference's stereo Frame constructor runs them (src/Frame.cc:113-125): two std::threads each
// calling ExtractORB -> ORBextractor::operator() on its own extractor, then ComputeStereoMatches.
// Checked against the CPU oracle (oracle/orbref.h, test infrastructure) frame after frame:
//   - keypoints and descriptors of both images (operator()'s outputs, ORBextractor.h:66-68);
//   - the public mvImagePyramid (ORBextractor.h:100) of BOTH extractors, all levels held at once
//     after both calls, each level against the oracle's level (the reader is
//     Frame::ComputeStereoMatches, Frame.cc:529,620-640); the oracle's CPU ComputeStereoMatches
//     run on the adapter's mvImagePyramid gives the oracle's own result;
//   - Frame_gpu.cc's ComputeStereoMatches (mvuRight / mvDepth) bit for bit.
// Built twice (tests/cpp/Makefile): default (host pyramid) and ORBFE_ADAPTER_GPU_STEREO=1 (no
// pyramid leaves the GPU; mvImagePyramid stays empty). Prints one "ADAPTER {json}" line with the
// p50 latency of operator() on one image and of the stereo Frame sequence, then OK / MISMATCH.
// Exit: 0 parity ok, 1 mismatch, 77 no GPU.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "Frame.h"
#include "ORBextractor.h"
#include "orbfe.hpp"
#include "orbfe_synth.h"
#include "../../oracle/orbref.h"

#ifndef ORBFE_ADAPTER_GPU_STEREO
#define ORBFE_ADAPTER_GPU_STEREO 0
#endif

namespace ORB_SLAM2 {
// src/Frame.cc:296-302
void Frame::ExtractORB(int flag, const cv::Mat& im) {
  if (flag == 0)
    (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors);
  else
    (*mpORBextractorRight)(im, cv::Mat(), mvKeysRight, mDescriptorsRight);
}
}  // namespace ORB_SLAM2

using ORB_SLAM2::Frame;
using ORB_SLAM2::ORBextractor;

namespace {
constexpr int kRows = 376, kCols = 1241, kLevels = 8;
constexpr float kFx = 718.856f, kCx = 607.1928f, kCy = 185.2157f, kBf = 386.1448f;

struct Ref {  // the oracle's results for one image
  std::vector<orbfe_keypoint> k;
  std::vector<uint8_t> d;
  std::vector<std::vector<uint8_t>> lv;
  int rows[kLevels], cols[kLevels];
};

Ref oracle_extract(const std::vector<uint8_t>& img) {
  Ref r;
  orbref_extractor* e = orbref_extractor_create(2000, 1.2f, kLevels, 20, 7);
  const int cap = 8000;
  r.k.resize(cap);
  r.d.resize((size_t)cap * 32);
  int n = 0;
  orbref_extract(e, img.data(), kRows, kCols, kCols, r.k.data(), cap, r.d.data(), &n);
  r.k.resize(n);
  r.d.resize((size_t)n * 32);
  r.lv.resize(kLevels);
  for (int l = 0; l < kLevels; l++) {
    orbref_get_level(e, l, nullptr, 0, &r.rows[l], &r.cols[l]);
    r.lv[l].resize((size_t)r.rows[l] * r.cols[l]);
    orbref_get_level(e, l, r.lv[l].data(), (int)r.lv[l].size(), &r.rows[l], &r.cols[l]);
  }
  orbref_extractor_destroy(e);
  return r;
}

int compare_features(const std::vector<cv::KeyPoint>& kg, const cv::Mat& dg, const Ref& r, const char* tag) {
  if (kg.size() != r.k.size()) {
    std::printf("%s: keypoint count %zu vs %zu\n", tag, kg.size(), r.k.size());
    return 1;
  }
  for (size_t i = 0; i < kg.size(); i++) {
    const cv::KeyPoint& a = kg[i];
    const orbfe_keypoint& b = r.k[i];
    if (a.pt.x != b.x || a.pt.y != b.y || a.size != b.size || a.response != b.response || a.octave != b.octave ||
        a.class_id != b.class_id || std::fabs(a.angle - b.angle) > 1e-5f) {
      std::printf("%s: keypoint %zu differs\n", tag, i);
      return 1;
    }
  }
  if (kg.empty()) return dg.empty() ? 0 : 1;  // operator() releases the Mat (ORBextractor.cc:1062-1063)
  if (dg.rows != (int)kg.size() || dg.cols != 32 || std::memcmp(dg.data, r.d.data(), r.d.size()) != 0) {
    std::printf("%s: descriptors differ\n", tag);
    return 1;
  }
  return 0;
}

#if !ORBFE_ADAPTER_GPU_STEREO
// every level of the extractor's mvImagePyramid against the oracle's, and no two levels overlap
int compare_pyramid(const std::vector<cv::Mat>& pyr, const Ref& r, const char* tag) {
  int fails = 0;
  if ((int)pyr.size() != kLevels) {
    std::printf("%s: mvImagePyramid has %zu levels\n", tag, pyr.size());
    return 1;
  }
  for (int l = 0; l < kLevels; l++) {
    const cv::Mat& m = pyr[l];
    if (m.rows != r.rows[l] || m.cols != r.cols[l] || m.step < (size_t)m.cols) {
      std::printf("%s: level %d shape %dx%d vs %dx%d\n", tag, l, m.rows, m.cols, r.rows[l], r.cols[l]);
      fails++;
      continue;
    }
    for (int y = 0; y < m.rows; y++)
      if (std::memcmp(m.data + (size_t)y * m.step, r.lv[l].data() + (size_t)y * m.cols, m.cols) != 0) {
        std::printf("%s: level %d row %d differs\n", tag, l, y);
        fails++;
        break;
      }
    for (int k = 0; k < l; k++) {  // [data, data + (rows-1)*step + cols) pairwise disjoint
      const uint8_t *a0 = pyr[k].data, *a1 = a0 + (size_t)(pyr[k].rows - 1) * pyr[k].step + pyr[k].cols;
      const uint8_t *b0 = m.data, *b1 = b0 + (size_t)(m.rows - 1) * m.step + m.cols;
      if (a0 < b1 && b0 < a1) {
        std::printf("%s: levels %d and %d alias\n", tag, k, l);
        fails++;
      }
    }
  }
  return fails;
}
#endif

void oracle_stereo(const std::vector<orbfe_keypoint>& kl, const std::vector<uint8_t>& dl,
                   const std::vector<orbfe_keypoint>& kr, const std::vector<uint8_t>& dr, const orbref_level_view* vl,
                   const orbref_level_view* vr, std::vector<float>& u, std::vector<float>& d) {
  orbref_extractor* e = orbref_extractor_create(2000, 1.2f, kLevels, 20, 7);
  std::vector<float> scale(kLevels), inv(kLevels), s2(kLevels), is2(kLevels);
  std::vector<int32_t> fpl(kLevels), umax(16);
  orbref_get_tables(e, scale.data(), inv.data(), s2.data(), is2.data(), fpl.data(), umax.data());
  orbref_extractor_destroy(e);
  u.assign(kl.size(), -1.f);
  d.assign(kl.size(), -1.f);
  orbref_compute_stereo_matches(kl.data(), dl.data(), (int)kl.size(), kr.data(), dr.data(), (int)kr.size(), vl, vr,
                                kLevels, scale.data(), inv.data(), kBf / kFx, kBf, u.data(), d.data());
}

double p50_ms(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
double time_ms(const std::function<void()>& f) {
  const auto t0 = std::chrono::steady_clock::now();
  f();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
  std::unique_ptr<ORBextractor> el, er;
  try {
    el.reset(new ORBextractor(2000, 1.2f, kLevels, 20, 7));
    er.reset(new ORBextractor(2000, 1.2f, kLevels, 20, 7));
  } catch (const orbfe::Error& e) {
    std::printf("no device: %s\n", e.what());
    return 77;
  }
  Frame F;
  F.mpORBextractorLeft = el.get();
  F.mpORBextractorRight = er.get();
  F.mK = cv::Mat(3, 3, CV_32F);
  std::memset(F.mK.data, 0, 9 * sizeof(float));
  F.mK.at<float>(0, 0) = kFx;
  F.mK.at<float>(1, 1) = kFx;
  F.mK.at<float>(0, 2) = kCx;
  F.mK.at<float>(1, 2) = kCy;
  F.mK.at<float>(2, 2) = 1.f;
  F.mbf = kBf;

  std::vector<uint8_t> left((size_t)kRows * kCols), right((size_t)kRows * kCols);
  auto stereo_frame = [&](const cv::Mat& L, const cv::Mat& R) {  // Frame.cc:113-125
    std::thread tl(&Frame::ExtractORB, &F, 0, std::cref(L));
    std::thread tr(&Frame::ExtractORB, &F, 1, std::cref(R));
    tl.join();
    tr.join();
    F.N = (int)F.mvKeys.size();
    F.ComputeStereoMatches();
  };
  int fails = 0, matched = 0;
  for (int t = 0; t < 3; t++) {  // three frames: every view must follow the latest call
    if (orbfe_synth_frame(11 + t, kRows, kCols, 0, left.data(), right.data(), kCols) != 0) return 1;
    const cv::Mat L(kRows, kCols, CV_8UC1, left.data(), kCols), R(kRows, kCols, CV_8UC1, right.data(), kCols);
    stereo_frame(L, R);
    const Ref rl = oracle_extract(left), rr = oracle_extract(right);
    fails += compare_features(F.mvKeys, F.mDescriptors, rl, "left");
    fails += compare_features(F.mvKeysRight, F.mDescriptorsRight, rr, "right");
    orbref_level_view vl[kLevels], vr[kLevels];
    for (int l = 0; l < kLevels; l++) {
      vl[l] = orbref_level_view{rl.lv[l].data(), rl.rows[l], rl.cols[l], rl.cols[l]};
      vr[l] = orbref_level_view{rr.lv[l].data(), rr.rows[l], rr.cols[l], rr.cols[l]};
    }
    std::vector<float> u_ref, d_ref;
    oracle_stereo(rl.k, rl.d, rr.k, rr.d, vl, vr, u_ref, d_ref);
#if !ORBFE_ADAPTER_GPU_STEREO
    // both extractors' levels, all held at once (the CPU ComputeStereoMatches reads left and
    // right levels of any octave in one pass)
    fails += compare_pyramid(el->mvImagePyramid, rl, "left pyramid");
    fails += compare_pyramid(er->mvImagePyramid, rr, "right pyramid");
    {  // the reference's CPU ComputeStereoMatches over the adapter's mvImagePyramid
      orbref_level_view al[kLevels], ar[kLevels];
      for (int l = 0; l < kLevels; l++) {
        const cv::Mat &a = el->mvImagePyramid[l], &b = er->mvImagePyramid[l];
        al[l] = orbref_level_view{a.data, a.rows, a.cols, (int)a.step};
        ar[l] = orbref_level_view{b.data, b.rows, b.cols, (int)b.step};
      }
      std::vector<float> u, d;
      oracle_stereo(rl.k, rl.d, rr.k, rr.d, al, ar, u, d);
      if (std::memcmp(u.data(), u_ref.data(), 4 * u.size()) != 0 || std::memcmp(d.data(), d_ref.data(), 4 * d.size()) != 0) {
        std::printf("frame %d: CPU ComputeStereoMatches over mvImagePyramid differs\n", t);
        fails++;
      }
    }
#else
    for (int l = 0; l < kLevels; l++)
      if (!el->mvImagePyramid[l].empty() || !er->mvImagePyramid[l].empty()) {
        std::printf("frame %d: mvImagePyramid[%d] populated in a GPU-stereo build\n", t, l);
        fails++;
      }
#endif
    // Frame_gpu.cc: ComputeStereoMatches on the device pyramids
    if (F.mvuRight.size() != u_ref.size() || std::memcmp(F.mvuRight.data(), u_ref.data(), 4 * u_ref.size()) != 0 ||
        std::memcmp(F.mvDepth.data(), d_ref.data(), 4 * d_ref.size()) != 0) {
      std::printf("frame %d: Frame::ComputeStereoMatches (GPU) differs\n", t);
      fails++;
    }
    for (float u : F.mvuRight) matched += u >= 0;
  }
  // latency: operator() on one image (one thread), and the stereo Frame sequence
  std::vector<double> t_op, t_frame;
  const cv::Mat L(kRows, kCols, CV_8UC1, left.data(), kCols), R(kRows, kCols, CV_8UC1, right.data(), kCols);
  std::vector<cv::KeyPoint> kps;
  cv::Mat desc;
  for (int i = 0; i < iters + 5; i++) {
    const double a = time_ms([&] { (*el)(L, cv::Mat(), kps, desc); });
    const double b = time_ms([&] { stereo_frame(L, R); });
    if (i >= 5) {
      t_op.push_back(a);
      t_frame.push_back(b);
    }
  }
  std::printf("ADAPTER {\"gpu_stereo_build\": %d, \"operator_p50_ms\": %.4f, \"stereo_frame_p50_ms\": %.4f, "
              "\"iters\": %d, \"stereo_matched_3_frames\": %d}\n",
              ORBFE_ADAPTER_GPU_STEREO, p50_ms(t_op), p50_ms(t_frame), iters, matched);
  std::printf("%s: %zu + %zu keypoints\n", fails ? "MISMATCH" : "OK", F.mvKeys.size(), F.mvKeysRight.size());
  return fails ? 1 : 0;
}
