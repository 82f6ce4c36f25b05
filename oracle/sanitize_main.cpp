// sanitize_main.cpp -- the oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5;
// TEST INFRASTRUCTURE ONLY). `make -C oracle sanitize` links this driver with the oracle sources and
// the synthetic-frame generator, all built -fsanitize=address,undefined; tests/test_oracle_sanitize.py
// runs it. It walks the hot path the parity tests use: extraction (KITTI, TUM and odd shapes, small
// and flat images, both resize modes), ComputeStereoMatches on two extractors' pyramids, the
// vocabulary transform (BowVector + FeatureVector), SearchForTriangulation and
// SearchByProjection(local). Exit 0 = clean (a sanitizer report aborts with a non-zero status).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../include/orbfe_synth.h"
#include "orbref.h"

namespace {

struct Extracted {
  std::vector<orbfe_keypoint> kp;
  std::vector<uint8_t> desc;
};

Extracted extract(orbref_extractor* h, const std::vector<uint8_t>& img, int rows, int cols) {
  Extracted e;
  const int cap = 2000 + 64 * 8 + 64;
  e.kp.resize(cap);
  e.desc.resize((size_t)cap * 32);
  int n = 0;
  const int st = orbref_extract(h, img.empty() ? nullptr : img.data(), rows, cols, (size_t)cols, e.kp.data(), cap,
                                 e.desc.data(), &n);
  if (st != 0) {
    std::printf("orbref_extract %dx%d: status %d\n", cols, rows, st);
    std::exit(1);
  }
  e.kp.resize(n);
  e.desc.resize((size_t)n * 32);
  return e;
}

std::vector<std::vector<uint8_t>> levels(orbref_extractor* h, int nlev, std::vector<orbref_level_view>& views) {
  std::vector<std::vector<uint8_t>> out(nlev);
  views.resize(nlev);
  for (int l = 0; l < nlev; l++) {
    int r = 0, c = 0;
    orbref_get_level(h, l, nullptr, 0, &r, &c);
    out[l].resize((size_t)r * c);
    orbref_get_level(h, l, out[l].data(), (int)out[l].size(), &r, &c);
    views[l] = orbref_level_view{out[l].data(), r, c, c};
  }
  return out;
}

}  // namespace

int main() {
  const int shapes[][2] = {{376, 1241}, {480, 640}, {301, 517}, {240, 320}};
  float scale[8], inv_scale[8], sigma2[8], inv_sigma2[8];
  int32_t nfeat[8], umax[16];
  std::mt19937 rng(7);
  for (int mode = 0; mode < 2; mode++) {
    for (auto& s : shapes) {
      const int rows = s[0], cols = s[1];
      orbref_extractor* el = orbref_extractor_create(2000, 1.2f, 8, 20, 7);
      orbref_extractor* er = orbref_extractor_create(2000, 1.2f, 8, 20, 7);
      orbref_set_resize_mode(el, mode);
      orbref_set_resize_mode(er, mode);
      orbref_get_tables(el, scale, inv_scale, sigma2, inv_sigma2, nfeat, umax);
      std::vector<uint8_t> l((size_t)rows * cols), r((size_t)rows * cols);
      orbfe_synth_frame(11 + mode, rows, cols, 0, l.data(), r.data(), cols);
      Extracted a = extract(el, l, rows, cols), b = extract(er, r, rows, cols);
      std::vector<orbref_level_view> vl, vr;
      auto pl = levels(el, 8, vl);
      auto pr = levels(er, 8, vr);
      std::vector<float> ur(a.kp.size() + 1), dep(a.kp.size() + 1);
      orbref_compute_stereo_matches(a.kp.data(), a.desc.data(), (int)a.kp.size(), b.kp.data(), b.desc.data(),
                                    (int)b.kp.size(), vl.data(), vr.data(), 8, scale, inv_scale, 0.537f,
                                    386.1448f, ur.data(), dep.data());
      // vocabulary: a random k=6 / L=3 tree, every leaf a word
      const int k = 6, L = 3;
      std::vector<int32_t> parent(1, -1);
      std::vector<uint8_t> leaf(1, 0);
      int first = 0, width = 1;
      for (int d = 1; d <= L; d++) {
        for (int p = first; p < first + width; p++)
          for (int c = 0; c < k; c++) {
            parent.push_back(p);
            leaf.push_back(d == L);
          }
        first += width;
        width *= k;
      }
      const int N = (int)parent.size();
      std::vector<uint8_t> nd((size_t)N * 32);
      for (auto& x : nd) x = (uint8_t)rng();
      std::vector<double> w(N);
      for (int i = 0; i < N; i++) w[i] = leaf[i] ? 0.5 + (rng() % 1000) / 100.0 : 0.0;
      orbref_vocab* voc = nullptr;
      if (orbref_vocab_from_table(N, k, L, 0, 0, parent.data(), leaf.data(), nd.data(), w.data(), &voc)) std::abort();
      std::vector<orbfe_feature_vector> fvs(2);
      std::vector<std::vector<uint32_t>> ids(2), words(2);
      std::vector<std::vector<int32_t>> offs(2), idx(2);
      std::vector<std::vector<double>> wts(2);
      const Extracted* ex[2] = {&a, &b};
      for (int s2 = 0; s2 < 2; s2++) {
        const int n = (int)ex[s2]->kp.size();
        ids[s2].resize(n + 1);
        offs[s2].resize(n + 2);
        idx[s2].resize(n + 1);
        words[s2].resize(n + 1);
        wts[s2].resize(n + 1);
        int nw = 0, nn = 0;
        orbref_vocab_transform_full(voc, ex[s2]->desc.data(), n, 1, words[s2].data(), wts[s2].data(), &nw,
                                    ids[s2].data(), offs[s2].data(), idx[s2].data(), &nn);
        fvs[s2] = orbfe_feature_vector{nn, ids[s2].data(), offs[s2].data(), idx[s2].data()};
      }
      orbref_vocab_free(voc);
      // SearchForTriangulation between the two sides
      std::vector<float> ur2(b.kp.size() + 1, -1.0f);
      std::vector<uint8_t> mp1(a.kp.size() + 1, 0), mp2(b.kp.size() + 1, 0);
      orbfe_frame_view f1{}, f2{};
      auto fill = [&](orbfe_frame_view& f, const Extracted& e, const float* u, const uint8_t* mp) {
        f.n = (int)e.kp.size();
        f.keys_un = e.kp.data();
        f.u_right = u;
        f.descriptors = e.desc.data();
        f.mp_state = mp;
        f.nlevels = 8;
        f.scale_factors = scale;
        f.level_sigma2 = sigma2;
        f.min_x = 0;
        f.max_x = (float)cols;
        f.min_y = 0;
        f.max_y = (float)rows;
        f.grid_inv_w = 64.0f / cols;
        f.grid_inv_h = 48.0f / rows;
        f.fx = f.fy = 718.856f;
        f.cx = cols / 2.0f;
        f.cy = rows / 2.0f;
        f.bf = 386.1448f;
        f.b = 0.537f;
      };
      fill(f1, a, ur.data(), mp1.data());
      fill(f2, b, ur2.data(), mp2.data());
      const float f12[9] = {0, -0.05f, 9.3f, 0.05f, 0, -610.f, -9.3f, 610.f, 0};
      std::vector<int32_t> m12(a.kp.size() + 1);
      int nm = 0;
      orbref_search_for_triangulation(&f1, &f2, &fvs[0], &fvs[1], f12, 620.f, 180.f, 0, 1, m12.data(), &nm);
      // SearchByProjection(local) with MapPoints on the left keypoints
      const int M = 3000;
      std::vector<uint8_t> fl(M), md((size_t)M * 32);
      std::vector<float> px(M), py(M), pxr(M), vc(M);
      std::vector<int32_t> lv(M), best(M);
      for (int i = 0; i < M; i++) {
        fl[i] = (uint8_t)(1u | ((rng() & 1) ? 4u : 0u));
        px[i] = (float)(rng() % cols);
        py[i] = (float)(rng() % rows);
        pxr[i] = px[i] - 10.0f;
        vc[i] = 0.9f;
        lv[i] = (int)(rng() % 8);
        for (int j = 0; j < 32; j++) md[(size_t)i * 32 + j] = (uint8_t)rng();
      }
      orbfe_local_mappoints mps{M, fl.data(), px.data(), py.data(), pxr.data(), lv.data(), vc.data(), md.data()};
      orbref_search_by_projection_local(&f1, &mps, 3.0f, 0.8f, best.data(), &nm);
      std::printf("mode %d %dx%d: %zu / %zu keypoints, %d local matches\n", mode, cols, rows, a.kp.size(),
                  b.kp.size(), nm);
      orbref_extractor_destroy(el);
      orbref_extractor_destroy(er);
    }
  }
  // degenerate inputs: a flat image (no corner anywhere) and a small 4-level one
  orbref_extractor* h = orbref_extractor_create(500, 1.2f, 4, 20, 7);
  extract(h, std::vector<uint8_t>((size_t)200 * 300, 128), 200, 300);
  std::vector<uint8_t> small((size_t)110 * 130);
  orbfe_synth_frame(3, 110, 130, 0, small.data(), nullptr, 130);
  extract(h, small, 110, 130);
  orbref_extractor_destroy(h);
  std::printf("OK\n");
  return 0;
}
