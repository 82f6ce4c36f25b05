// trig_check.cpp -- TEST INFRASTRUCTURE (oracle), not product code. Pins the cos / sin of the
// descriptor steering angle.
//
// ORBextractor.cc:66 has `using namespace std;`, so ORBextractor.cc:110 `(float)cos(angle)` with
// a float `angle` resolves to std::cos(float), i.e. glibc cosf / sinf -- which are NOT correctly
// rounded: (float)cos((double)x) differs from glibc's cosf / sinf for 1,484,894 of the float
// degree values in [0, 360) on glibc 2.35. The oracle therefore calls cosf / sinf (orbref.cpp),
// and k_describe runs a port of glibc's algorithm. This file restates that algorithm once more
// (glibc 2.35 sysdeps/ieee754/flt-32 sinf / cosf, |x| < 120, the FMA ifunc variant that x86-64
// CPUs with FMA run: constants and operation order read from libm's __cosf_fma / __sinf_fma) and
// checks restatement and GPU against glibc over every float the steering can see: angle =
// fastAtan2(...) * factorPI (:109) with fastAtan2 in [0, 360) degrees.
//
//   orbref_trig_mismatch  glibc cosf / sinf vs the restatement below, per degree value
//   orbref_trig_compare   glibc cosf / sinf vs cos / sin arrays computed elsewhere (the GPU)
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace {

const float kFactorPi = (float)(M_PI / 180.f);  // ORBextractor.cc:107

inline float bits_to_float(uint32_t b) {
  float f;
  memcpy(&f, &b, 4);
  return f;
}
inline uint32_t float_to_bits(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}

// __sincosf_table[0] (table 1 negates the c coefficients) and the quadrant signs
const double kC0 = 1.0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
             kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
const double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
const double kHpiInv = 0x1.45f306dc9c883p+23, kHpi = 0x1.921fb54442d18p+0;
const double kSign[4] = {1.0, -1.0, -1.0, 1.0};

double cos_poly(double x2) {  // sinf_poly, cos branch, table 0
  const double x4 = x2 * x2;
  const double c1 = fma(x2, kC1, kC0);
  const double c2 = fma(x2, kC4, kC3);
  const double x6 = x2 * x4;
  const double c = fma(x4, kC2, c1);
  return fma(c2, x6, c);
}
double sin_poly(double x, double x2) {  // sinf_poly, sin branch
  const double s1 = fma(x2, kS3, kS2);
  const double x3 = x2 * x;
  const double x5 = x3 * x2;
  const double s = fma(x3, kS1, x);
  return fma(s1, x5, s);
}
// cosf (want_sin = false) / sinf (true) for 0 <= y < 120
float sincosf_restated(float y, bool want_sin) {
  uint32_t bits;
  memcpy(&bits, &y, 4);
  const uint32_t top12 = (bits >> 20) & 0x7ff;
  const double x = y;
  if (top12 <= 0x3f3) {  // |y| < 0.75 (abstop12 < abstop12(pi/4))
    if (top12 <= 0x397) return want_sin ? y : 1.0f;  // |y| < 2^-12
    const double x2 = x * x;
    return (float)(want_sin ? sin_poly(x, x2) : cos_poly(x2));
  }
  const int n = ((int)(x * kHpiInv) + 0x800000) >> 24;  // reduce_fast: truncate, then round
  const double r = fma(-(double)n, kHpi, x);
  const double r2 = r * r;
  const bool sin_branch = ((n & 1) == 0) == want_sin;
  if (sin_branch) return (float)sin_poly(r * kSign[n & 3], r2);
  const double c = cos_poly(r2);
  return (float)((n & 2) ? -c : c);
}

template <class F>
uint64_t parallel_count(uint64_t n, int nthreads, F&& body) {
  nthreads = std::max(1, std::min(nthreads, 256));
  std::atomic<uint64_t> total{0};
  std::vector<std::thread> pool;
  const uint64_t per = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    const uint64_t b = per * t, e = std::min(n, b + per);
    if (b >= e) break;
    pool.emplace_back([&, b, e] { total += body(b, e); });
  }
  for (auto& th : pool) th.join();
  return total.load();
}

}  // namespace

extern "C" {

// Degree values with bit patterns [deg_bits_begin, deg_bits_end) stepping by `stride`: the number
// whose glibc cosf or sinf of (deg * factorPI) differs from the restatement above; the smallest
// such bit pattern goes to *first_bad (0xffffffff if none).
uint64_t orbref_trig_mismatch(uint32_t deg_bits_begin, uint32_t deg_bits_end, uint32_t stride,
                              int nthreads, uint32_t* first_bad) {
  if (stride == 0) stride = 1;
  const uint64_t n = deg_bits_end > deg_bits_begin ? (deg_bits_end - deg_bits_begin + stride - 1) / stride : 0;
  std::atomic<uint32_t> first{0xffffffffu};
  const uint64_t bad = parallel_count(n, nthreads, [&](uint64_t b, uint64_t e) {
    uint64_t c = 0;
    for (uint64_t i = b; i < e; i++) {
      const uint32_t bits = deg_bits_begin + (uint32_t)(i * stride);
      const float ang = bits_to_float(bits) * kFactorPi;
      const bool ok = float_to_bits(cosf(ang)) == float_to_bits(sincosf_restated(ang, false)) &&
                      float_to_bits(sinf(ang)) == float_to_bits(sincosf_restated(ang, true));
      if (!ok) {
        c++;
        uint32_t f = first.load();
        while (bits < f && !first.compare_exchange_weak(f, bits)) {
        }
      }
    }
    return c;
  });
  if (first_bad) *first_bad = first.load();
  return bad;
}

// cos_vals / sin_vals[i] computed elsewhere for degree bit pattern deg_bits_begin + i: the count
// that differ from glibc cosf / sinf of (deg * factorPI); the first differing index goes to
// *first_bad (UINT64_MAX if none).
uint64_t orbref_trig_compare(uint32_t deg_bits_begin, uint64_t n, const float* cos_vals,
                             const float* sin_vals, int nthreads, uint64_t* first_bad) {
  std::atomic<uint64_t> first{UINT64_MAX};
  const uint64_t bad = parallel_count(n, nthreads, [&](uint64_t b, uint64_t e) {
    uint64_t c = 0;
    for (uint64_t i = b; i < e; i++) {
      const float ang = bits_to_float(deg_bits_begin + (uint32_t)i) * kFactorPi;
      const bool ok = float_to_bits(cosf(ang)) == float_to_bits(cos_vals[i]) &&
                      float_to_bits(sinf(ang)) == float_to_bits(sin_vals[i]);
      if (!ok) {
        c++;
        uint64_t f = first.load();
        while (i < f && !first.compare_exchange_weak(f, i)) {
        }
      }
    }
    return c;
  });
  if (first_bad) *first_bad = first.load();
  return bad;
}

}  // extern "C"
