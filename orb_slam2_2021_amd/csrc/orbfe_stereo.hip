// orbfe_stereo.hip -- Frame::ComputeStereoMatches (src/Frame.cc:522-700) for gfx950.
//
// Three launches per batch of rectified pairs, all reading the pyramids and keypoints the
// extractor left resident in HBM:
//   k_stereo_rows    one block per pair: counting sort of the right keypoints into (octave,
//                    floor(y)) buckets (CSR) with each keypoint's packed row span (Frame.cc:532-548).
//   k_stereo_match   16 lanes per left keypoint: the Hamming search over the row band
//                    (:557-607), then the 11x11 SAD sweep over 11 shifts -- lane = window row --
//                    and the parabola fit / disparity test (:609-684).
//   k_stereo_median  one block per pair: radix-select of the median SAD and the 2.1x-median
//                    rejection (:686-699).
// The reference's row table lists, for row v, the right keypoints whose [floor(y-r), ceil(y+r)]
// span covers v, in iR order, and keeps the first minimum. Here right keypoints are bucketed by
// (octave, floor(y)); the candidates of a level-L keypoint on row v are the bucket rows of octaves
// L-1..L+1 within each octave's band, filtered by that exact span test, and ties are broken by the
// smallest iR -- the same winner.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_stereo.h"
#include "orbfe_device.h"
#include "orbfe_internal.h"
#include "orbfe_ktimer.h"

namespace {

constexpr int ST_W = 5;   // half window (Frame.cc:617)
constexpr int ST_L = 5;   // half shift range (:627)
constexpr int ST_TH_ORB = (100 + 50) / 2;  // thOrbDist = (TH_HIGH + TH_LOW) / 2 (:527)
constexpr int ST_TAB_MAX = 16384;          // LDS bucket table bound (ints)

struct StereoGeom {
  const uint8_t* pyrL;  // left / right pyramids (may be the same handle's)
  const uint8_t* pyrR;
  long long strideL, strideR;
  int pL0, pR0;         // pair p: left pyramid image pL0 + p, right pyramid image pR0 + p
  int kL0, kR0;         // pair p: keypoints / descriptors / counts of images kL0 + p, kR0 + p
  int cap, nlevels, rows0;
  int nbk;  // octave buckets: nlevels (bucket per octave and row) or 1 (per row only)
  float mbf, maxD;
  int w[ORBFE_MAX_LEVELS], pitch[ORBFE_MAX_LEVELS];
  int h[ORBFE_MAX_LEVELS];
  int rbo[ORBFE_MAX_LEVELS];  // row band of each octave bucket (see launch code)
  long long off[ORBFE_MAX_LEVELS];
  float scale[ORBFE_MAX_LEVELS], inv_scale[ORBFE_MAX_LEVELS];
};

// ---- k_stereo_rows ----------------------------------------------------------------------------
// 256 threads: the rows table runs on the matching stream beside the extraction kernels, where
// smaller workgroups find room sooner (1024 threads measured no faster; 1024-thread workgroups of
// k_vocab measured -3.7 %)
constexpr int ROWS_THREADS = 256;

// Counting sort of pair p's right keypoints into buckets (octave, floor(y)); bucket entry
// {x bits, (minr & 0xffff) | maxr << 16, octave, iR} with minr/maxr as Frame.cc:543-544.
__global__ __launch_bounds__(ROWS_THREADS) void k_stereo_rows(StereoGeom g, const orbfe_keypoint* __restrict__ kps,
                                                              const int32_t* __restrict__ counts,
                                                              int32_t* __restrict__ row_start,
                                                              uint4* __restrict__ buckets) {
  extern __shared__ int s_hist[];  // nbk*(rows0+1) counters, then 16 ints of scan scratch
  const int ntab = g.nbk * (g.rows0 + 1);
  int* wsum = s_hist + ntab;
  const int p = blockIdx.x, t = threadIdx.x;
  const int img = g.kR0 + p;
  const int nR = min(counts[img], g.cap);
  const orbfe_keypoint* K = kps + (long long)img * g.cap;
  for (int r = t; r < ntab; r += ROWS_THREADS) s_hist[r] = 0;
  __syncthreads();
  auto bucket = [&](float y, int oct) {
    const int row = min(max((int)floorf(y), 0), g.rows0 - 1);
    return (g.nbk > 1 ? oct * (g.rows0 + 1) : 0) + row;
  };
  for (int i = t; i < nR; i += ROWS_THREADS) atomicAdd(&s_hist[bucket(K[i].y, K[i].octave)], 1);
  __syncthreads();
  block_scan_excl(s_hist, ntab, wsum);
  int32_t* rs = row_start + (long long)p * ntab;
  for (int r = t; r < ntab; r += ROWS_THREADS) rs[r] = s_hist[r];
  __syncthreads();
  uint4* B = buckets + (long long)p * g.cap;
  for (int i = t; i < nR; i += ROWS_THREADS) {
    const float x = K[i].x, y = K[i].y;
    const int oct = K[i].octave;
    const int slot = atomicAdd(&s_hist[bucket(y, oct)], 1);
    const float r = 2.0f * g.scale[oct];
    const int maxr = (int)ceilf(y + r);
    const int minr = (int)floorf(y - r);
    B[slot] = make_uint4(__float_as_uint(x), ((unsigned)minr & 0xffffu) | ((unsigned)maxr << 16),
                         (unsigned)oct, (unsigned)i);
  }
}

// ---- median filter ---------------------------------------------------------------------------
// median = the (M/2)-th smallest SAD of the M matches (:686-688); SADs are < 2^16 (121 * 510), so
// two 8-bit radix-select passes find it. Every match with SAD >= 1.5*1.4*median is dropped.
__device__ __forceinline__ void select_bin(const int* hist, int k, int* s_out, int* wsum) {
  // the bin b with prefix(b) <= k < prefix(b+1): block-wide inclusive scan of 256 bins
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const int hv = hist[t];
  int inc = hv;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  for (int q = 0; q < w; q++) inc += wsum[q];
  const int exc = inc - hv;
  if (exc <= k && k < inc) {
    s_out[0] = t;
    s_out[1] = k - exc;
  }
  __syncthreads();
}

struct MedianSmem {
  int hist[256];
  int wsum[4];
  int sel[3];
};

// Runs on the 256 threads of one block over pair p's SADs (sad_in[i] < 0: no match).
__device__ void median_filter(MedianSmem& sm, int nL, const int32_t* S, float* ur, float* dep) {
  const int t = threadIdx.x;
  if (t == 0) sm.sel[2] = 0;
  sm.hist[t] = 0;
  __syncthreads();
  int m = 0;
  for (int i = t; i < nL; i += 256) {
    const int s = S[i];
    if (s >= 0) {
      m++;
      atomicAdd(&sm.hist[(s >> 8) & 255], 1);
    }
  }
  m = wave_sum(m);
  if (lane_id() == 0) atomicAdd(&sm.sel[2], m);
  __syncthreads();
  const int M = sm.sel[2];
  if (M == 0) return;  // the reference indexes an empty vector here; nothing is rejected
  select_bin(sm.hist, M / 2, sm.sel, sm.wsum);
  const int hb = sm.sel[0], k2 = sm.sel[1];
  sm.hist[t] = 0;
  __syncthreads();
  for (int i = t; i < nL; i += 256) {
    const int s = S[i];
    if (s >= 0 && (s >> 8) == hb) atomicAdd(&sm.hist[s & 255], 1);
  }
  __syncthreads();
  select_bin(sm.hist, k2, sm.sel, sm.wsum);
  const float median = (float)((hb << 8) | sm.sel[0]);
  const float thDist = 1.5f * 1.4f * median;
  for (int i = t; i < nL; i += 256) {
    const int s = S[i];
    if (s >= 0 && !((float)s < thDist)) {
      ur[i] = -1.0f;
      dep[i] = -1.0f;
    }
  }
}

// ---- k_stereo_match ---------------------------------------------------------------------------
// DPP within the 16-lane row that holds one keypoint
__device__ __forceinline__ unsigned row_sum16(unsigned v) {
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);  // row_ror:2
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);  // row_ror:1
  return v;
}
__device__ __forceinline__ unsigned row_bcast5(unsigned v) {  // lane 5 of the row to all 16
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x155, 0xf, 0xf, false);  // row_newbcast:5
}
__device__ __forceinline__ unsigned long long group16_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    const unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ unsigned byte_at(const uint32_t* a, int k) { return (a[k >> 2] >> (8 * (k & 3))) & 255u; }
// u16 pair (byte k, byte k+1) of a little-endian byte string held in dwords
__device__ __forceinline__ unsigned pair_at(const uint32_t* a, int k) {
  const int w = k >> 2, b = k & 3;
  if (b == 0) return __builtin_amdgcn_perm(0u, a[w], 0x0c010c00u);
  if (b == 1) return __builtin_amdgcn_perm(0u, a[w], 0x0c020c01u);
  if (b == 2) return __builtin_amdgcn_perm(0u, a[w], 0x0c030c02u);
  return __builtin_amdgcn_perm(a[w + 1], a[w], 0x0c040c03u);
}

__device__ __forceinline__ void stereo_one(const StereoGeom& g, const orbfe_keypoint* __restrict__ kps,
                                           const uint8_t* __restrict__ desc, const int32_t* __restrict__ row_start,
                                           const uint4* __restrict__ buckets, float* __restrict__ u_right,
                                           float* __restrict__ depth, int32_t* __restrict__ sad_out, int p, int i,
                                           int j, int imgL, int imgR) {
  const int pimgL = g.pL0 + p, pimgR = g.pR0 + p;
  const orbfe_keypoint kpL = kps[(long long)imgL * g.cap + i];
  const long long o = (long long)p * g.cap + i;
  float ur_out = -1.0f, dep_out = -1.0f;
  int sad_best = -1;
  const float vL = kpL.y, uL = kpL.x;
  const int levelL = kpL.octave;
  const float minU = uL - g.maxD, maxU = uL - 0.0f;  // minD = 0 (:552-575)
  if (vL >= 0.0f && vL < (float)g.rows0 && !(maxU < 0)) {
    const int v = (int)vL;
    // candidate ranges: the bucket rows of octaves levelL-1..levelL+1 that can hold a right
    // keypoint whose row span covers v (one range of all octaves when nbk == 1)
    const int ntab = g.nbk * (g.rows0 + 1);
    const int32_t* rs = row_start + (long long)p * ntab;
    int b0 = 0, n0 = 0, b1 = 0, n1 = 0, b2 = 0, n2 = 0;
    auto range = [&](int ob, int& b, int& n) {
      const int rb = g.rbo[ob];
      const int lo = max(0, v - rb), hi = min(g.rows0 - 1, v + rb);
      const int base = ob * (g.rows0 + 1);
      b = rs[base + lo];
      n = rs[base + hi + 1] - b;
    };
    if (g.nbk > 1) {
      if (levelL - 1 >= 0) range(levelL - 1, b0, n0);
      range(levelL, b1, n1);
      if (levelL + 1 < g.nlevels) range(levelL + 1, b2, n2);
    } else {
      range(0, b1, n1);
    }
    uint4 dl0, dl1;
    load_desc(desc + ((long long)imgL * g.cap + i) * 32, dl0, dl1);
    const uint4* B = buckets + (long long)p * g.cap;
    const uint8_t* DR = desc + (long long)imgR * g.cap * 32;
    unsigned long long best = ~0ull;
    const int total = n0 + n1 + n2;
    for (int k = j; k < total; k += 16) {
      const int idx = k < n0 ? b0 + k : (k < n0 + n1 ? b1 + (k - n0) : b2 + (k - n0 - n1));
      const uint4 e = B[idx];
      const int minr = (int)(int16_t)(e.y & 0xffffu), maxr = (int)e.y >> 16;
      const int oct = (int)e.z;
      const float uR = __uint_as_float(e.x);
      if (v >= minr && v <= maxr && oct >= levelL - 1 && oct <= levelL + 1 && uR >= minU && uR <= maxU) {
        uint4 d0, d1;
        load_desc(DR + (long long)e.w * 32, d0, d1);
        const int dist = hamming256(dl0, dl1, d0, d1);
        if (dist < 100) {  // bestDist starts at TH_HIGH (:578); ties: smallest iR (first in :586)
          const unsigned long long key = ((unsigned long long)dist << 32) | e.w;
          best = key < best ? key : best;
        }
      }
    }
    best = group16_min_u64(best);
    const int bestDist = best == ~0ull ? 100 : (int)(best >> 32);
    if (bestDist < ST_TH_ORB) {
      const int iR = (int)(best & 0xffffffffu);
      const float uR0 = kps[(long long)imgR * g.cap + iR].x;
      const float sf = g.inv_scale[levelL];
      const float scaleduL = roundf(kpL.x * sf);
      const float scaledvL = roundf(kpL.y * sf);
      const float scaleduR0 = roundf(uR0 * sf);
      const float iniu = scaleduR0 + ST_L - ST_W;
      const float endu = scaleduR0 + ST_L + ST_W + 1;
      const int yL = (int)scaledvL, xL = (int)scaleduL, xR0 = (int)scaleduR0;
      const int cols = g.w[levelL], rows = g.h[levelL];
      // :633-635, plus the windows OpenCV's rowRange/colRange would reject (never on extractor
      // output; the oracle skips them the same way)
      const bool ok = !(iniu < 0 || endu >= cols) && yL - ST_W >= 0 && yL + ST_W < rows &&
                      xL - ST_W >= 0 && xL + ST_W < cols && xR0 - ST_L - ST_W >= 0;
      if (ok) {
        // lane j = window row j (lanes 11..15 re-read row 10 and contribute nothing)
        const int row = yL + min(j, 2 * ST_W) - ST_W;
        const uint8_t* pl = g.pyrL + (long long)pimgL * g.strideL + g.off[levelL] +
                            (long long)row * g.pitch[levelL] + (xL - ST_W);
        const uint8_t* pr = g.pyrR + (long long)pimgR * g.strideR + g.off[levelL] +
                            (long long)row * g.pitch[levelL] + (xR0 - ST_L - ST_W);
        const uint32_t* ql = reinterpret_cast<const uint32_t*>((uintptr_t)pl & ~(uintptr_t)3);
        const uint32_t* qr = reinterpret_cast<const uint32_t*>((uintptr_t)pr & ~(uintptr_t)3);
        const int sl = (int)((uintptr_t)pl & 3), sr = (int)((uintptr_t)pr & 3);
        uint32_t wl[4], wr[7], al[4], ar[7];
#pragma unroll
        for (int k = 0; k < 4; k++) wl[k] = ql[k];
#pragma unroll
        for (int k = 0; k < 7; k++) wr[k] = qr[k];
#pragma unroll
        for (int k = 0; k < 3; k++) al[k] = __builtin_amdgcn_alignbyte(wl[k + 1], wl[k], sl);
        al[3] = 0;
#pragma unroll
        for (int k = 0; k < 6; k++) ar[k] = __builtin_amdgcn_alignbyte(wr[k + 1], wr[k], sr);
        ar[6] = 0;
        // |(IL - IL(w,w)) - (IR - IR(w,w))| = |(IL + IR(w,w)) - (IR + IL(w,w))|, all terms in
        // [0, 510]: packed u16 pairs through v_sad_u16 (2 columns per instruction)
        const unsigned cL = row_bcast5(byte_at(al, ST_W));
        const unsigned cL2 = cL | (cL << 16);
        unsigned Lp[6];
#pragma unroll
        for (int k = 0; k < 5; k++) Lp[k] = pair_at(al, 2 * k);
        Lp[5] = byte_at(al, 10);  // column 10 alone (hi half 0)
        unsigned Bp[21];           // Bp[c] = (IR[c] + cL, IR[c+1] + cL), c = 0..20
#pragma unroll
        for (int c = 0; c < 21; c++) Bp[c] = pair_at(ar, c) + cL2;
        unsigned acc[2 * ST_L + 1];
#pragma unroll
        for (int s = 0; s < 2 * ST_L + 1; s++) {
          const unsigned cR = row_bcast5(byte_at(ar, s + ST_W));
          const unsigned cR2 = cR | (cR << 16);
          unsigned a = 0;
#pragma unroll
          for (int k = 0; k < 5; k++) a = __builtin_amdgcn_sad_u16(Lp[k] + cR2, Bp[s + 2 * k], a);
          a = __builtin_amdgcn_sad_u16(Lp[5] + cR, Bp[s + 10] & 0xffffu, a);
          acc[s] = j <= 2 * ST_W ? a : 0u;
        }
        // per-shift totals (< 2^16: 121 * 510) two to a dword, summed over the 16 lanes
        unsigned tot[2 * ST_L + 1];
#pragma unroll
        for (int t2 = 0; t2 < ST_L; t2++) {
          const unsigned q = row_sum16(acc[2 * t2] | (acc[2 * t2 + 1] << 16));
          tot[2 * t2] = q & 0xffffu;
          tot[2 * t2 + 1] = q >> 16;
        }
        tot[2 * ST_L] = row_sum16(acc[2 * ST_L]);
        // cv::norm(NORM_L1) of integer-valued windows is exact; strict < keeps the first minimum
        int best_sad = 0x7fffffff, bestinc = 0;
#pragma unroll
        for (int s = 0; s < 2 * ST_L + 1; s++)
          if ((float)tot[s] < (float)best_sad) {
            best_sad = (int)tot[s];
            bestinc = s - ST_L;
          }
        if (bestinc != -ST_L && bestinc != ST_L) {
          float d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
          for (int s = 1; s < 2 * ST_L; s++)
            if (s == bestinc + ST_L) {
              d1 = (float)tot[s - 1];
              d2 = (float)tot[s];
              d3 = (float)tot[s + 1];
            }
          const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));  // :661
          if (!(deltaR < -1 || deltaR > 1)) {
            float bestuR = g.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
            float disparity = uL - bestuR;
            if (disparity >= 0.0f && disparity < g.maxD) {
              if (disparity <= 0) {
                disparity = (float)0.01;
                bestuR = (float)((double)uL - 0.01);
              }
              dep_out = g.mbf / disparity;
              ur_out = bestuR;
              sad_best = best_sad;
            }
          }
        }
      }
    }
  }
  if (j == 0) {
    u_right[o] = ur_out;
    depth[o] = dep_out;
    sad_out[o] = sad_best;
  }
}

__global__ __launch_bounds__(256) void k_stereo_match(StereoGeom g, const orbfe_keypoint* __restrict__ kps,
                                                      const uint8_t* __restrict__ desc,
                                                      const int32_t* __restrict__ counts,
                                                      const int32_t* __restrict__ row_start,
                                                      const uint4* __restrict__ buckets,
                                                      float* __restrict__ u_right, float* __restrict__ depth,
                                                      int32_t* __restrict__ sad_out) {
  const int2 blk = xcd_block2d();
  const int p = blk.y;
  const int j = threadIdx.x & 15;
  const int i = blk.x * 16 + (threadIdx.x >> 4);
  const int imgL = g.kL0 + p, imgR = g.kR0 + p;
  const int nL = min(counts[imgL], g.cap);
  if (i < nL) stereo_one(g, kps, desc, row_start, buckets, u_right, depth, sad_out, p, i, j, imgL, imgR);
}

// One block per pair. (A last-block-done tail in k_stereo_match would save this launch, but on
// MI355X the agent-scope release/acquire it needs writes back and invalidates the per-XCD L2 in
// every block: measured 413 us vs 30 + 8 us for the two launches.)
__global__ __launch_bounds__(256) void k_stereo_median(int left0, int cap, const int32_t* __restrict__ counts,
                                                       const int32_t* __restrict__ sad_in,
                                                       float* __restrict__ u_right, float* __restrict__ depth) {
  __shared__ MedianSmem sm;
  const int p = blockIdx.x;
  const long long base = (long long)p * cap;
  median_filter(sm, min(counts[left0 + p], cap), sad_in + base, u_right + base, depth + base);
}

}  // namespace

// ---- scratch owned by the extractor handle ------------------------------------------------------
struct OrbfeStereoScratch {
  int32_t* d_row_start = nullptr;
  size_t row_start_n = 0;
  uint4* d_buckets = nullptr;
  int32_t* d_sad = nullptr;
  size_t slots_n = 0;
  // host-buffer entry points
  orbfe_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  int32_t* d_counts = nullptr;
  float* d_out = nullptr;
  size_t io_n = 0;
  uint8_t* h_stage = nullptr;
  size_t h_stage_n = 0;
};

void orbfe_internal_stereo_free(OrbfeStereoScratch* s) {
  if (!s) return;
  hipFree(s->d_row_start);
  hipFree(s->d_buckets);
  hipFree(s->d_sad);
  hipFree(s->d_kps);
  hipFree(s->d_desc);
  hipFree(s->d_counts);
  hipFree(s->d_out);
  if (s->h_stage) hipHostFree(s->h_stage);
  delete s;
}

static OrbfeStereoScratch* scratch_of(orbfe_extractor* h) {
  OrbfeStereoScratch** slot = orbfe_internal_stereo_slot(h);
  if (!*slot) *slot = new OrbfeStereoScratch();
  return *slot;
}

// The three launches for n_pairs pairs: left pyramid image pl0 + p of PL, right pyramid image
// pr0 + p of PR, keypoints / descriptors / counts of images kl0 + p and kr0 + p of d_kps (cap
// slots per image), outputs at p*cap.
static int launch_stereo(OrbfeStereoScratch* S, const OrbfePyramid& PL, int pl0, const OrbfePyramid& PR,
                         int pr0, int n_pairs, int kl0, int kr0, const orbfe_keypoint* d_kps,
                         const uint8_t* d_desc, const int32_t* d_counts, int cap, float mbf, float mb,
                         float* d_u_right, float* d_depth, hipStream_t s) {
  if (PL.nlevels != PR.nlevels)
    return orbfe_set_error(ORBFE_ERR_ARG, "left and right extractors differ in levels");
  for (int l = 0; l < PL.nlevels; l++)
    if (PL.w[l] != PR.w[l] || PL.h[l] != PR.h[l] || PL.pitch[l] != PR.pitch[l] || PL.off[l] != PR.off[l] ||
        PL.scale[l] != PR.scale[l])
      return orbfe_set_error(ORBFE_ERR_ARG, "left and right pyramids differ in geometry");
  const size_t rs_n = (size_t)n_pairs * PL.nlevels * (PL.h[0] + 1), sl_n = (size_t)n_pairs * cap;
  if (rs_n > S->row_start_n) {
    hipFree(S->d_row_start);
    S->d_row_start = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&S->d_row_start, rs_n * sizeof(int32_t)));
    S->row_start_n = rs_n;
  }
  if (sl_n > S->slots_n) {
    hipFree(S->d_buckets);
    hipFree(S->d_sad);
    S->d_buckets = nullptr;
    S->d_sad = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&S->d_buckets, sl_n * sizeof(uint4)));
    ORBFE_HIP_CHECK(hipMalloc(&S->d_sad, sl_n * sizeof(int32_t)));
    S->slots_n = sl_n;
  }
  StereoGeom g;
  std::memset(&g, 0, sizeof(g));
  g.pyrL = PL.base;
  g.pyrR = PR.base;
  g.strideL = PL.image_stride;
  g.strideR = PR.image_stride;
  g.pL0 = pl0;
  g.pR0 = pr0;
  g.kL0 = kl0;
  g.kR0 = kr0;
  g.cap = cap;
  g.nlevels = PL.nlevels;
  g.rows0 = PL.h[0];
  g.mbf = mbf;
  const float minZ = mb;
  g.maxD = mbf / minZ;  // :553
  for (int l = 0; l < PL.nlevels; l++) {
    g.w[l] = PL.w[l];
    g.h[l] = PL.h[l];
    g.pitch[l] = PL.pitch[l];
    g.off[l] = PL.off[l];
    g.scale[l] = PL.scale[l];
    g.inv_scale[l] = PL.inv_scale[l];
  }
  // Row band of a bucket: a right keypoint at row floor(y) = b of octave o covers v only if
  // floor(y - r) <= v <= ceil(y + r), r = 2 scale[o] (:541-544), i.e. |b - v| <= ceil(r) + 1;
  // one more row absorbs the float rounding of y -+ r.
  g.nbk = PL.nlevels * (g.rows0 + 1) <= ST_TAB_MAX ? PL.nlevels : 1;
  if (g.nbk == 1 && g.rows0 + 1 > ST_TAB_MAX)
    return orbfe_set_error(ORBFE_ERR_ARG, "image taller than the stereo row table");
  int rb_all = 0;
  for (int l = 0; l < PL.nlevels; l++) {
    g.rbo[l] = (int)std::ceil(2.0f * PL.scale[l]) + 2;
    rb_all = std::max(rb_all, g.rbo[l]);
  }
  if (g.nbk == 1) g.rbo[0] = rb_all;
  const size_t lds = sizeof(int) * (g.nbk * (g.rows0 + 1) + 16);
  ORBFE_LAUNCH("k_stereo_rows", k_stereo_rows, dim3(n_pairs), dim3(ROWS_THREADS), lds, s, g, d_kps, d_counts,
                     S->d_row_start, S->d_buckets);
  ORBFE_HIP_CHECK(hipGetLastError());
  ORBFE_LAUNCH("k_stereo_match", k_stereo_match, dim3((cap + 15) / 16, n_pairs), dim3(256), 0, s, g, d_kps, d_desc,
                     d_counts, S->d_row_start, S->d_buckets, d_u_right, d_depth, S->d_sad);
  ORBFE_HIP_CHECK(hipGetLastError());
  ORBFE_LAUNCH("k_stereo_median", k_stereo_median, dim3(n_pairs), dim3(256), 0, s, kl0, cap, d_counts, S->d_sad,
                     d_u_right, d_depth);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

extern "C" int orbfe_compute_stereo_matches_batch_device(orbfe_extractor* h, int n_pairs, int left0,
                                                         int right0, const orbfe_keypoint* d_kps,
                                                         const uint8_t* d_desc, const int32_t* d_counts,
                                                         int cap, float mbf, float mb, float* d_u_right,
                                                         float* d_depth, void* stream) {
  if (!h || n_pairs < 0 || cap <= 0 || !d_kps || !d_desc || !d_counts || !d_u_right || !d_depth)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_stereo_matches_batch_device: bad argument");
  if (n_pairs == 0) return ORBFE_OK;
  OrbfePyramid P;
  int st = orbfe_internal_pyramid(h, &P);
  if (st != ORBFE_OK) return st;
  if (left0 < 0 || right0 < 0 || left0 + n_pairs > P.n_images || right0 + n_pairs > P.n_images)
    return orbfe_set_error(ORBFE_ERR_ARG, "stereo pair images outside the last extract call");
  if (cap < P.total_key_slots) return orbfe_set_error(ORBFE_ERR_CAPACITY, "cap < orbfe_max_keypoints");
  hipSetDevice(P.device);
  hipStream_t s = stream ? (hipStream_t)stream : P.stream;
  return launch_stereo(scratch_of(h), P, left0, P, right0, n_pairs, left0, right0, d_kps, d_desc, d_counts,
                       cap, mbf, mb, d_u_right, d_depth, s);
}

static int ensure_io(OrbfeStereoScratch* S, size_t slots) {
  if (slots > S->io_n) {
    hipFree(S->d_kps);
    hipFree(S->d_desc);
    hipFree(S->d_counts);
    hipFree(S->d_out);
    if (S->h_stage) hipHostFree(S->h_stage);
    S->d_kps = nullptr;
    S->d_desc = nullptr;
    S->d_counts = nullptr;
    S->d_out = nullptr;
    S->h_stage = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&S->d_kps, 2 * slots * sizeof(orbfe_keypoint)));
    ORBFE_HIP_CHECK(hipMalloc(&S->d_desc, 2 * slots * 32));
    ORBFE_HIP_CHECK(hipMalloc(&S->d_counts, 2 * sizeof(int32_t)));
    ORBFE_HIP_CHECK(hipMalloc(&S->d_out, 2 * slots * sizeof(float)));
    ORBFE_HIP_CHECK(hipHostMalloc(&S->h_stage, 2 * slots * (sizeof(orbfe_keypoint) + 32 + sizeof(float)) + 64));
    S->io_n = slots;
  }
  return ORBFE_OK;
}

extern "C" int orbfe_compute_stereo_matches(orbfe_extractor* h_left, int image_left,
                                            orbfe_extractor* h_right, int image_right,
                                            const orbfe_keypoint* kps_l, const uint8_t* desc_l, int n_l,
                                            const orbfe_keypoint* kps_r, const uint8_t* desc_r, int n_r,
                                            float mbf, float mb, float* u_right, float* depth) {
  if (!h_left || !h_right || n_l < 0 || n_r < 0 || (n_l > 0 && (!kps_l || !desc_l || !u_right || !depth)) ||
      (n_r > 0 && (!kps_r || !desc_r)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_stereo_matches: bad argument");
  for (int i = 0; i < n_l; i++) u_right[i] = depth[i] = -1.0f;  // :524-525
  if (n_l == 0) return ORBFE_OK;
  OrbfePyramid PL, PR;
  int st = orbfe_internal_pyramid(h_left, &PL);
  if (st != ORBFE_OK) return st;
  st = orbfe_internal_pyramid(h_right, &PR);
  if (st != ORBFE_OK) return st;
  if (image_left < 0 || image_left >= PL.n_images || image_right < 0 || image_right >= PR.n_images)
    return orbfe_set_error(ORBFE_ERR_ARG, "stereo image outside the last extract call");
  if (PL.device != PR.device) return orbfe_set_error(ORBFE_ERR_ARG, "left and right handles on different devices");
  hipSetDevice(PL.device);
  if (h_right != h_left) ORBFE_HIP_CHECK(hipStreamSynchronize(PR.stream));  // right pyramid complete
  const int cap = std::max(PL.total_key_slots, std::max(n_l, n_r));
  OrbfeStereoScratch* S = scratch_of(h_left);
  st = ensure_io(S, (size_t)cap);
  if (st != ORBFE_OK) return st;
  // stage both keypoint / descriptor sets (slot 0 = left, slot 1 = right) in one H2D burst each
  orbfe_keypoint* hk = reinterpret_cast<orbfe_keypoint*>(S->h_stage);
  uint8_t* hd = S->h_stage + 2 * (size_t)cap * sizeof(orbfe_keypoint);
  std::memcpy(hk, kps_l, sizeof(orbfe_keypoint) * n_l);
  if (n_r) std::memcpy(hk + cap, kps_r, sizeof(orbfe_keypoint) * n_r);
  std::memcpy(hd, desc_l, (size_t)n_l * 32);
  if (n_r) std::memcpy(hd + (size_t)cap * 32, desc_r, (size_t)n_r * 32);
  int32_t* hc = reinterpret_cast<int32_t*>(hd + 2 * (size_t)cap * 32);
  hc[0] = n_l;
  hc[1] = n_r;
  hipStream_t s = PL.stream;
  ORBFE_HIP_CHECK(hipMemcpyAsync(S->d_kps, hk, 2 * (size_t)cap * sizeof(orbfe_keypoint), hipMemcpyHostToDevice, s));
  ORBFE_HIP_CHECK(hipMemcpyAsync(S->d_desc, hd, 2 * (size_t)cap * 32, hipMemcpyHostToDevice, s));
  ORBFE_HIP_CHECK(hipMemcpyAsync(S->d_counts, hc, 2 * sizeof(int32_t), hipMemcpyHostToDevice, s));
  st = launch_stereo(S, PL, image_left, PR, image_right, 1, 0, 1, S->d_kps, S->d_desc, S->d_counts, cap, mbf,
                     mb, S->d_out, S->d_out + cap, s);
  if (st != ORBFE_OK) return st;
  ORBFE_HIP_CHECK(hipStreamSynchronize(s));  // the staging area is reused for the results
  float* ho = reinterpret_cast<float*>(hk);
  ORBFE_HIP_CHECK(hipMemcpyAsync(ho, S->d_out, sizeof(float) * n_l, hipMemcpyDeviceToHost, s));
  ORBFE_HIP_CHECK(hipMemcpyAsync(ho + n_l, S->d_out + cap, sizeof(float) * n_l, hipMemcpyDeviceToHost, s));
  ORBFE_HIP_CHECK(hipStreamSynchronize(s));
  std::memcpy(u_right, ho, sizeof(float) * n_l);
  std::memcpy(depth, ho + n_l, sizeof(float) * n_l);
  return ORBFE_OK;
}

extern "C" int orbfe_stereo_frame(orbfe_extractor* h, const uint8_t* left, const uint8_t* right, int rows,
                                  int cols, size_t step, float mbf, float mb, orbfe_keypoint* kps_l,
                                  uint8_t* desc_l, int* n_l, orbfe_keypoint* kps_r, uint8_t* desc_r, int* n_r,
                                  int cap, float* u_right, float* depth) {
  if (!h || !left || !right || !n_l || !n_r)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_stereo_frame: bad argument");
  *n_l = *n_r = 0;
  if (rows == 0 || cols == 0) return ORBFE_OK;  // N = 0: the constructor returns early (:120-121)
  const int K = orbfe_max_keypoints(h, rows, cols);
  if (K < 0) return K;
  if (cap < K) return orbfe_set_error(ORBFE_ERR_CAPACITY, "cap < orbfe_max_keypoints");
  if (!kps_l || !desc_l || !kps_r || !desc_r || !u_right || !depth)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_stereo_frame: null output buffer");
  // ExtractORB(0) and ExtractORB(1) as one batch (:113-116); ComputeStereoMatches enqueued right
  // behind the extraction on the handle's stream, its uRight / depth copied down with the keypoints
  // (one wait for the whole Frame; the kernels see the keypoint counts on the device)
  const uint8_t* imgs[2] = {left, right};
  orbfe_keypoint* const kp_img[2] = {kps_l, kps_r};  // the results go straight to the caller's arrays
  uint8_t* const desc_img[2] = {desc_l, desc_r};
  int32_t counts[2] = {0, 0};
  float* ho = nullptr;
  auto stereo = [&]() -> int {
    OrbfePyramid P;
    int r = orbfe_internal_pyramid(h, &P);
    if (r != ORBFE_OK) return r;
    OrbfeStereoScratch* S = scratch_of(h);
    r = ensure_io(S, (size_t)K);
    if (r != ORBFE_OK) return r;
    r = launch_stereo(S, P, 0, P, 1, 1, 0, 1, P.io_kps, P.io_desc, P.io_counts, K, mbf, mb, S->d_out, S->d_out + K,
                      P.stream);
    if (r != ORBFE_OK) return r;
    ho = reinterpret_cast<float*>(S->h_stage);
    ORBFE_HIP_CHECK(hipMemcpyAsync(ho, S->d_out, sizeof(float) * 2 * (size_t)K, hipMemcpyDeviceToHost, P.stream));
    return ORBFE_OK;
  };
  const int st = orbfe_internal_extract_batch(h, 2, imgs, rows, cols, step, nullptr, nullptr, cap, counts, stereo,
                                              kp_img, desc_img);
  if (st != ORBFE_OK) return st;
  *n_l = counts[0];
  *n_r = counts[1];
  if (counts[0] == 0) return ORBFE_OK;
  std::memcpy(u_right, ho, sizeof(float) * counts[0]);
  std::memcpy(depth, ho + K, sizeof(float) * counts[0]);
  return ORBFE_OK;
}
