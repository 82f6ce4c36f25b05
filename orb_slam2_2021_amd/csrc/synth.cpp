// synth.cpp -- seeded synthetic KITTI-shaped grayscale frames.
//
// The reference's benchmark input (KITTI 00 stereo PNGs) is not available offline, so every
// benchmark and parity test runs on this generator. Image i of a sequence uses seed
// 0x0B5EED00 ^ i: splitmix64 seeds a xoshiro128** stream. Content: a smooth sinusoidal field,
// a layer of random rectangles composited in order (the corner-rich part FAST responds to), and
// sum-of-4-uniforms noise (sigma ~= 3). The right image of a stereo pair sees the same scene
// shifted left by d(y) = 8 + 32*y/H pixels, with independent noise.
#include <algorithm>
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

// ---- driving sequence (SURVEY 8(d) C3 KeyFrame pairs: frame t and t+1, poses step_z apart along z)
//
// A world of fronto-parallel textured billboards. Depth slab k (world z in [k, k+1) m) holds
// kSeqPerSlab billboards drawn from seed (seq_seed, k): centre x in +-70 m, y in +-21 m, width and
// height 0.3-2.5 m, an intensity, and for half of them an inner panel (inset by a quarter) of a
// second intensity. Frame t's left camera sits at (0, 0, t * step_z) looking down +z (pinhole fx,
// fy, cx, cy); the right camera of the pair is `baseline` metres to the right. Billboards between
// kSeqNear and kSeqFar metres ahead are painted far to near over the sinusoidal background at
// infinity (the same field as orbfe_synth_frame, zero disparity), then sum-of-4-uniforms noise
// (sigma ~= 3) seeded per (frame, side). The epipole of two consecutive left frames is (cx, cy):
// inside the image, so SearchForTriangulation's epipole gate (ORBmatcher.cc:757-763) is live.
namespace {
constexpr int kSeqPerSlab = 160;
constexpr float kSeqNear = 6.0f, kSeqFar = 80.0f;

struct Billboard {
  float z, x, y, hw, hh;
  int v, v_in;  // v_in < 0: no inner panel
};

void slab_billboards(uint64_t seq_seed, int64_t k, std::vector<Billboard>& out) {
  Xoshiro128ss g(seq_seed * 0x9E3779B97F4A7C15ull ^ (uint64_t)(k + 0x5EEDull) * 0xD1B54A32D192ED03ull);
  for (int i = 0; i < kSeqPerSlab; i++) {
    Billboard b;
    b.z = (float)k + g.uniform();
    b.x = -70.f + 140.f * g.uniform();
    b.y = -21.f + 42.f * g.uniform();
    b.hw = 0.5f * (0.3f + 2.2f * g.uniform());
    b.hh = 0.5f * (0.3f + 2.2f * g.uniform());
    b.v = g.range(0, 255);
    b.v_in = (g.next() & 1u) ? g.range(0, 255) : -1;
    out.push_back(b);
  }
}

// pixel columns [a, b) whose centres lie in [u0, u1)
inline void span(float u0, float u1, int n, int& a, int& b) {
  a = (int)std::ceil(u0 - 0.5f);
  b = (int)std::ceil(u1 - 0.5f);
  a = std::max(a, 0);
  b = std::min(b, n);
}

void render_sequence(const std::vector<Billboard>& bbs, float cam_x, float cam_z, int rows, int cols,
                     float fx, float fy, float cx, float cy, uint64_t noise_seed, uint8_t* out, size_t step) {
  Scene bg(0x0B5EED00ull, rows, cols, 0);  // the background field only (no rectangles)
  std::vector<float> img((size_t)rows * cols);
  for (int y = 0; y < rows; y++) bg.row(y, 0, img.data() + (size_t)y * cols);
  for (const Billboard& b : bbs) {  // far to near
    const float d = b.z - cam_z;
    if (d < kSeqNear || d >= kSeqFar) continue;
    const float sx = fx / d, sy = fy / d, u = cx + (b.x - cam_x) * sx, v = cy + b.y * sy;
    int x0, x1, y0, y1;
    span(u - b.hw * sx, u + b.hw * sx, cols, x0, x1);
    span(v - b.hh * sy, v + b.hh * sy, rows, y0, y1);
    for (int y = y0; y < y1; y++)
      for (int x = x0; x < x1; x++) img[(size_t)y * cols + x] = (float)b.v;
    if (b.v_in >= 0) {
      span(u - 0.5f * b.hw * sx, u + 0.5f * b.hw * sx, cols, x0, x1);
      span(v - 0.5f * b.hh * sy, v + 0.5f * b.hh * sy, rows, y0, y1);
      for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) img[(size_t)y * cols + x] = (float)b.v_in;
    }
  }
  Xoshiro128ss g(noise_seed);
  const float k = 3.0f * 1.7320508f;
  for (int y = 0; y < rows; y++)
    for (int x = 0; x < cols; x++) {
      float n = g.uniform() + g.uniform() + g.uniform() + g.uniform() - 2.0f;
      float v = std::nearbyint(img[(size_t)y * cols + x] + k * n);
      out[(size_t)y * step + x] = (uint8_t)(v < 0.f ? 0.f : (v > 255.f ? 255.f : v));
    }
}
}  // namespace

extern "C" int orbfe_synth_sequence_frame(uint64_t seq_seed, long long t, int rows, int cols, float fx, float fy,
                                          float cx, float cy, float baseline, float step_z, uint8_t* left,
                                          uint8_t* right, size_t step) {
  if (rows <= 0 || cols <= 0 || step < (size_t)cols || (!left && !right) || t < 0 || !(fx > 0.f) ||
      !(fy > 0.f) || !(step_z >= 0.f))
    return -1;
  const float cam_z = (float)((double)t * step_z);
  std::vector<Billboard> bbs;
  for (int64_t k = (int64_t)std::floor(cam_z + kSeqNear); k <= (int64_t)std::ceil(cam_z + kSeqFar); k++)
    slab_billboards(seq_seed, k, bbs);
  std::stable_sort(bbs.begin(), bbs.end(), [](const Billboard& a, const Billboard& b) { return a.z > b.z; });
  const uint64_t ns = (seq_seed ^ 0x5E0F5E0F5E0F5E0Full) + (uint64_t)t * 0x9E3779B97F4A7C15ull;
  if (left) render_sequence(bbs, 0.f, cam_z, rows, cols, fx, fy, cx, cy, ns ^ 0x1111111111111111ull, left, step);
  if (right)
    render_sequence(bbs, baseline, cam_z, rows, cols, fx, fy, cx, cy, ns ^ 0x2222222222222222ull, right, step);
  return 0;
}
