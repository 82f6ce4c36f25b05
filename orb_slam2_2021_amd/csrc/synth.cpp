// synth.cpp -- seeded synthetic KITTI-shaped grayscale frames.
//
// The reference's benchmark input (KITTI 00 stereo PNGs) is not available offline, so every
// benchmark and parity test runs on this generator. Image i of a sequence uses seed
// 0x0B5EED00 ^ i: splitmix64 seeds a xoshiro128** stream. Content: a smooth sinusoidal field,
// a layer of random rectangles composited in order (the corner-rich part FAST responds to), and
// sum-of-4-uniforms noise (sigma ~= 3). The right image of a stereo pair sees the same scene
// shifted left by d(y) = 8 + 32*y/H pixels, with independent noise.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/orbfe_synth.h"

namespace {
struct Xoshiro128ss {
  uint32_t s[4];
  explicit Xoshiro128ss(uint64_t seed) {
    for (int i = 0; i < 2; i++) {  // splitmix64
      uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      s[2 * i] = (uint32_t)z;
      s[2 * i + 1] = (uint32_t)(z >> 32);
    }
  }
  static uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
  uint32_t next() {
    const uint32_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 9;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 11);
    return r;
  }
  float uniform() { return (float)(next() >> 8) * (1.0f / 16777216.0f); }
  int range(int lo, int hi) { return lo + (int)(next() % (uint32_t)(hi - lo + 1)); }
};

struct Rect {
  int x0, y0, x1, y1, v;
};

struct Scene {
  float lx, ly;
  std::vector<Rect> rects;
  int cols, rows;
  Scene(uint64_t seed, int rows_, int cols_, int n_rects) : cols(cols_), rows(rows_) {
    Xoshiro128ss g(seed);
    lx = 150.f + 100.f * g.uniform();
    ly = 100.f + 100.f * g.uniform();
    rects.reserve(n_rects);
    for (int i = 0; i < n_rects; i++) {
      Rect r;
      int w = g.range(4, 64), h = g.range(4, 64);
      r.x0 = g.range(-16, cols + 40);  // scene extends right of the frame for the stereo shift
      r.y0 = g.range(-16, rows - 1);
      r.x1 = r.x0 + w;
      r.y1 = r.y0 + h;
      r.v = g.range(0, 255);
      rects.push_back(r);
    }
  }
  void row(int y, int x_shift, float* out) const {  // scene value at (x + x_shift, y)
    const float two_pi = 6.28318530717958647692f;
    const float cy = std::cos(two_pi * (float)y / ly);
    for (int x = 0; x < cols; x++) {
      int xs = x + x_shift;
      out[x] = 128.f + 50.f * std::sin(two_pi * (float)xs / lx) * cy;
    }
    for (const Rect& r : rects) {
      if (y < r.y0 || y >= r.y1) continue;
      int a = r.x0 - x_shift, b = r.x1 - x_shift;
      if (a < 0) a = 0;
      if (b > cols) b = cols;
      for (int x = a; x < b; x++) out[x] = (float)r.v;
    }
  }
};

void render(const Scene& sc, uint64_t noise_seed, int stereo_shift, uint8_t* out, size_t step) {
  Xoshiro128ss g(noise_seed);
  std::vector<float> row(sc.cols);
  const float k = 3.0f * 1.7320508f;  // sum of 4 U[0,1) has sd 1/sqrt(3): scale to sigma 3
  for (int y = 0; y < sc.rows; y++) {
    int shift = stereo_shift ? 8 + (32 * y) / sc.rows : 0;
    sc.row(y, shift, row.data());
    for (int x = 0; x < sc.cols; x++) {
      float n = g.uniform() + g.uniform() + g.uniform() + g.uniform() - 2.0f;
      float v = std::nearbyint(row[x] + k * n);
      out[(size_t)y * step + x] = (uint8_t)(v < 0.f ? 0.f : (v > 255.f ? 255.f : v));
    }
  }
}
}  // namespace

extern "C" int orbfe_synth_frame(uint64_t index, int rows, int cols, int n_rects, uint8_t* left,
                                 uint8_t* right, size_t step) {
  if (rows <= 0 || cols <= 0 || step < (size_t)cols || (!left && !right)) return -1;
  const uint64_t seed = 0x0B5EED00ull ^ index;
  Scene sc(seed, rows, cols, n_rects > 0 ? n_rects : ORBFE_SYNTH_DEFAULT_RECTS);
  if (left) render(sc, seed ^ 0x1111111111111111ull, 0, left, step);
  if (right) render(sc, seed ^ 0x2222222222222222ull, 1, right, step);
  return 0;
}
