// orbfe_device.h -- device helpers shared by the extractor and matcher kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// The whole library is compiled with -ffp-contract=off: every float expression below rounds each
// operation exactly like the reference's scalar x86 code.

#define ORBFE_WAVE 64

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }
// wave-uniform, so that per-wave indices derived from it stay in SGPRs (scalar loads and address math)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
__device__ __forceinline__ uint64_t lanemask_lt() {
  return (1ull << (unsigned)lane_id()) - 1ull;
}
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return (uint64_t)__ballot(p ? 1 : 0); }
// set bits of `mask` below this lane: v_mbcnt_lo + v_mbcnt_hi (2 VALU ops, mask from SGPRs)
__device__ __forceinline__ int prefix_in_wave(uint64_t mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// cvRound(float): round half to even (v_rndne_f32)
__device__ __forceinline__ int cv_round_f(float v) { return (int)__builtin_rintf(v); }

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:1672-1688) = popcount of the 256-bit xor.
__device__ __forceinline__ int hamming256(const uint4 a0, const uint4 a1, const uint4 b0,
                                          const uint4 b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}
__device__ __forceinline__ void load_desc(const uint8_t* p, uint4& d0, uint4& d1) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  d0 = q[0];
  d1 = q[1];
}

// OpenCV fastAtan2 (atanImpl<float>) in degrees; constants are computed on the host in float
// exactly as OpenCV's static initialisers do and passed in.
struct AtanConsts {
  float p1, p3, p5, p7, eps;
};
__device__ __forceinline__ float fast_atan2_dev(float y, float x, const AtanConsts& k) {
  float ax = fabsf(x), ay = fabsf(y), a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + k.eps);
    c2 = c * c;
    a = (((k.p7 * c2 + k.p5) * c2 + k.p3) * c2 + k.p1) * c;
  } else {
    c = ax / (ay + k.eps);
    c2 = c * c;
    a = 90.f - (((k.p7 * c2 + k.p5) * c2 + k.p3) * c2 + k.p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// Exclusive scan of data[0..n) in place by a 256-thread workgroup (4 waves); returns the total.
// wsum: 4 ints of LDS. Contains __syncthreads(): call from uniform control flow only.
// XCD-aware block remap (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"; observed
// round-robin dealing of blocks over the 8 XCDs). Returns the logical (x, y) block of a 2-D grid
// such that each XCD receives one contiguous range of logical blocks (x fastest): neighbouring
// cells / keypoints of one image then share an L2. Bijective for any grid size. Speed only.
__device__ __forceinline__ int2 xcd_block2d() {
  const int nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * gridDim.x + blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  return make_int2(id % gridDim.x, id / gridDim.x);
}

// LDS visibility among the lanes of one wavefront (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Exclusive scan of data[0..n) in LDS by the NT threads of the block (wsum: NT / 64 ints).
template <int NT>
__device__ inline int block_scan_excl_n(int* data, int n, int* wsum) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const int per = (n + NT - 1) / NT;
  const int beg = min(t * per, n), end = min(beg + per, n);
  int s = 0;
  for (int i = beg; i < end; i++) s += data[i];
  int inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int woff = 0, total = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) {
    woff += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  int run = woff + inc - s;
  for (int i = beg; i < end; i++) {
    const int v = data[i];
    data[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}
__device__ inline int block_scan_excl(int* data, int n, int* wsum) { return block_scan_excl_n<256>(data, n, wsum); }

// Three exclusive scans at once (one pair of barriers instead of three); wsum holds 3 x NT / 64 ints.
template <int NT>
__device__ inline int3 block_scan_excl3_n(int* a, int* b, int* c, int n, int* wsum) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  if (n <= 64) {  // (n is block-uniform) one wavefront scans, one barrier publishes
    if (w == 0) {
      const int va = lane < n ? a[lane] : 0, vb = lane < n ? b[lane] : 0, vc = lane < n ? c[lane] : 0;
      int ia = va, ib = vb, ic = vc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int ya = __shfl_up(ia, o, 64), yb = __shfl_up(ib, o, 64), yc = __shfl_up(ic, o, 64);
        if (lane >= o) {
          ia += ya;
          ib += yb;
          ic += yc;
        }
      }
      if (lane < n) {
        a[lane] = ia - va;
        b[lane] = ib - vb;
        c[lane] = ic - vc;
      }
      if (lane == 63) {
        wsum[0] = ia;
        wsum[1] = ib;
        wsum[2] = ic;
      }
    }
    __syncthreads();
    return make_int3(wsum[0], wsum[1], wsum[2]);
  }
  const int per = (n + NT - 1) / NT;
  const int beg = min(t * per, n), end = min(beg + per, n);
  int sa = 0, sb = 0, sc = 0;
  for (int i = beg; i < end; i++) {
    sa += a[i];
    sb += b[i];
    sc += c[i];
  }
  int ia = sa, ib = sb, ic = sc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int ya = __shfl_up(ia, o, 64), yb = __shfl_up(ib, o, 64), yc = __shfl_up(ic, o, 64);
    if (lane >= o) {
      ia += ya;
      ib += yb;
      ic += yc;
    }
  }
  if (lane == 63) {
    wsum[w] = ia;
    wsum[NW + w] = ib;
    wsum[2 * NW + w] = ic;
  }
  __syncthreads();
  int oa = 0, ob = 0, oc = 0, ta = 0, tb = 0, tc = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) {
    const int xa = wsum[k], xb = wsum[NW + k], xc = wsum[2 * NW + k];
    if (k < w) {
      oa += xa;
      ob += xb;
      oc += xc;
    }
    ta += xa;
    tb += xb;
    tc += xc;
  }
  int ra = oa + ia - sa, rb = ob + ib - sb, rc = oc + ic - sc;
  for (int i = beg; i < end; i++) {
    const int va = a[i], vb = b[i], vc = c[i];
    a[i] = ra;
    b[i] = rb;
    c[i] = rc;
    ra += va;
    rb += vb;
    rc += vc;
  }
  __syncthreads();
  return make_int3(ta, tb, tc);
}
__device__ inline int3 block_scan_excl3(int* a, int* b, int* c, int n, int* wsum) {
  return block_scan_excl3_n<256>(a, b, c, n, wsum);
}

// Exclusive scan of data[0..n) in LDS by the 1024 threads of the block (wsum: 16 ints).
__device__ inline void block_scan_excl_1024(int* data, int n, int* wsum) {
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const int per = (n + 1023) / 1024;
  const int beg = min(t * per, n), end = min(beg + per, n);
  int s = 0;
  for (int i = beg; i < end; i++) s += data[i];
  int inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int run = inc - s;
  for (int q = 0; q < w; q++) run += wsum[q];
  for (int i = beg; i < end; i++) {
    const int v = data[i];
    data[i] = run;
    run += v;
  }
  __syncthreads();
}

#define ORBFE_HIP_CHECK(expr)                                     \
  do {                                                            \
    hipError_t _e = (expr);                                       \
    if (_e != hipSuccess) return orbfe_set_hip_error(_e, #expr); \
  } while (0)

int orbfe_set_error(int code, const char* msg);
int orbfe_set_hip_error(hipError_t e, const char* what);
