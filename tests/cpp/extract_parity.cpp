// C++ caller of liborbfe.so through include/orbfe.hpp, the way a reference-side adapter would
// call it: one orbfe::Extractor per thread, operator() on 8-bit images, then the matcher.
// Checks every result against the CPU oracle's C API (oracle/orbref.h, test infrastructure).
// Exit: 0 parity ok, 1 mismatch, 77 no GPU (orbfe error on create).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/orbfe.hpp"
#include "../../include/orbfe_synth.h"
#include "../../oracle/orbref.h"

static int compare(const std::vector<orbfe::KeyPoint>& kg, const std::vector<uint8_t>& dg,
                   const std::vector<orbfe_keypoint>& kr, const std::vector<uint8_t>& dr, const char* tag) {
  if (kg.size() != kr.size()) {
    std::printf("%s: keypoint count %zu vs %zu\n", tag, kg.size(), kr.size());
    return 1;
  }
  for (size_t i = 0; i < kg.size(); i++) {
    const orbfe_keypoint &a = kg[i], &b = kr[i];
    if (a.x != b.x || a.y != b.y || a.size != b.size || a.response != b.response || a.octave != b.octave ||
        a.class_id != b.class_id || std::fabs(a.angle - b.angle) > 1e-5f) {
      std::printf("%s: keypoint %zu differs\n", tag, i);
      return 1;
    }
  }
  if (dg != dr) {
    std::printf("%s: descriptors differ\n", tag);
    return 1;
  }
  return 0;
}

int main() {
  const int rows = 376, cols = 1241;
  std::vector<uint8_t> left((size_t)rows * cols), right((size_t)rows * cols);
  if (orbfe_synth_frame(3, rows, cols, 0, left.data(), right.data(), cols) != 0) return 1;
  try {
    orbfe::Extractor probe(2000, 1.2f, 8, 20, 7);
  } catch (const orbfe::Error& e) {
    std::printf("no device: %s\n", e.what());
    return 77;
  }
  // two extractor instances on two threads, as Frame.cc:113-116 runs the stereo pair
  orbfe::Extractor el(2000, 1.2f, 8, 20, 7), er(2000, 1.2f, 8, 20, 7);
  std::vector<orbfe::KeyPoint> kl, kr;
  std::vector<uint8_t> dl, dr;
  std::thread tl([&] { el(left.data(), rows, cols, cols, kl, dl); });
  std::thread tr([&] { er(right.data(), rows, cols, cols, kr, dr); });
  tl.join();
  tr.join();

  orbref_extractor* ref = orbref_extractor_create(2000, 1.2f, 8, 20, 7);
  int fails = 0;
  const std::vector<uint8_t>* imgs[2] = {&left, &right};
  const std::vector<orbfe::KeyPoint>* gk[2] = {&kl, &kr};
  const std::vector<uint8_t>* gd[2] = {&dl, &dr};
  for (int s = 0; s < 2; s++) {
    const int cap = 4000;
    std::vector<orbfe_keypoint> k(cap);
    std::vector<uint8_t> d((size_t)cap * 32);
    int n = 0;
    if (orbref_extract(ref, imgs[s]->data(), rows, cols, cols, k.data(), cap, d.data(), &n) != 0) return 1;
    k.resize(n);
    d.resize((size_t)n * 32);
    fails += compare(*gk[s], *gd[s], k, d, s ? "right" : "left");
  }
  // mvImagePyramid level views of the left image match the oracle's levels
  {
    std::vector<orbfe_keypoint> k(4000);
    std::vector<uint8_t> d(4000 * 32);
    int n = 0;
    orbref_extract(ref, left.data(), rows, cols, cols, k.data(), 4000, d.data(), &n);
    for (int l = 0; l < 8; l++) {
      orbfe::LevelView v = el.level(l);
      int r = 0, c = 0;
      orbref_get_level(ref, l, nullptr, 0, &r, &c);
      std::vector<uint8_t> lv((size_t)r * c);
      orbref_get_level(ref, l, lv.data(), (int)lv.size(), &r, &c);
      if (v.rows != r || v.cols != c) {
        std::printf("level %d shape\n", l);
        fails++;
        continue;
      }
      for (int y = 0; y < r; y++)
        if (std::memcmp(v.data + (size_t)y * v.step, lv.data() + (size_t)y * c, c) != 0) {
          std::printf("level %d row %d differs\n", l, y);
          fails++;
          break;
        }
    }
  }
  orbref_extractor_destroy(ref);
  // Frame::ComputeStereoMatches over the two extractors' pyramids vs the oracle on the oracle's
  {
    const float bf = 386.1448f, mb = bf / 718.856f;
    std::vector<float> ur, dep;
    orbfe::ComputeStereoMatches(el, er, kl, dl, kr, dr, bf, mb, ur, dep);
    orbref_extractor* rl = orbref_extractor_create(2000, 1.2f, 8, 20, 7);
    orbref_extractor* rr = orbref_extractor_create(2000, 1.2f, 8, 20, 7);
    std::vector<orbfe_keypoint> k(4000);
    std::vector<uint8_t> d(4000 * 32);
    int n = 0;
    orbref_extract(rl, left.data(), rows, cols, cols, k.data(), 4000, d.data(), &n);
    orbref_extract(rr, right.data(), rows, cols, cols, k.data(), 4000, d.data(), &n);
    std::vector<std::vector<uint8_t>> lvl(16);
    orbref_level_view vl[8], vr[8];
    for (int l = 0; l < 8; l++)
      for (int side = 0; side < 2; side++) {
        orbref_extractor* e = side ? rr : rl;
        int r = 0, c = 0;
        orbref_get_level(e, l, nullptr, 0, &r, &c);
        std::vector<uint8_t>& buf = lvl[2 * l + side];
        buf.resize((size_t)r * c);
        orbref_get_level(e, l, buf.data(), (int)buf.size(), &r, &c);
        (side ? vr : vl)[l] = orbref_level_view{buf.data(), r, c, c};
      }
    std::vector<float> scale(8), inv(8), s2(8), is2(8);
    std::vector<int32_t> fpl(8), umax(16);
    orbref_get_tables(rl, scale.data(), inv.data(), s2.data(), is2.data(), fpl.data(), umax.data());
    std::vector<float> wu(kl.size()), wd(kl.size());
    orbref_compute_stereo_matches(kl.data(), dl.data(), (int)kl.size(), kr.data(), dr.data(), (int)kr.size(), vl,
                                  vr, 8, scale.data(), inv.data(), mb, bf, wu.data(), wd.data());
    int matched = 0;
    for (size_t i = 0; i < kl.size(); i++) {
      if (std::memcmp(&ur[i], &wu[i], 4) != 0 || std::memcmp(&dep[i], &wd[i], 4) != 0) {
        std::printf("stereo: keypoint %zu differs (%g %g vs %g %g)\n", i, ur[i], dep[i], wu[i], wd[i]);
        fails++;
        break;
      }
      matched += ur[i] >= 0;
    }
    std::printf("stereo: %d of %zu left keypoints matched\n", matched, kl.size());
    orbref_extractor_destroy(rl);
    orbref_extractor_destroy(rr);
  }
  // DescriptorDistance on the extracted descriptors
  for (size_t i = 0; i + 1 < kl.size() && i < 64; i++)
    if (orbfe::Matcher::DescriptorDistance(&dl[i * 32], &dl[(i + 1) * 32]) !=
        orbref_descriptor_distance(&dl[i * 32], &dl[(i + 1) * 32]))
      fails++;
  std::printf("%s: %zu + %zu keypoints\n", fails ? "MISMATCH" : "OK", kl.size(), kr.size());
  return fails ? 1 : 0;
}
