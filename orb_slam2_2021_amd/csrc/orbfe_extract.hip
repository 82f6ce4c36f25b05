// orbfe_extract.hip -- ORBextractor::operator() as six CDNA4 kernels (gfx950, wave64).
//
// Reference: src/ORBextractor.cc of lreithmayr/ORB_SLAM2_2021 (operator() :1041-1103).
// Pipeline per batch of same-shaped images, all on one HIP stream:
//   k_copy0                   the caller's image -> level 0 of the padded pyramid block
//   k_resize   x (nlevels-1)  ComputePyramid :1105-1135 -- one launch per level (level l reads the
//                             rounded uint8 level l-1, exactly the reference chain), 11-bit fixed
//                             point bilinear with OpenCV's SIMD128 vertical rounding (Appendix A.3)
//   k_fast                    the FAST half of ComputeKeyPointsOctTree :792-832 -- one wavefront per
//                             ~30x30 cell ROI staged in LDS: 9-of-16 arc strength per pixel, strict
//                             3x3 NMS inside the cell, iniTh -> minTh fallback, row-major compaction
//                             with wave ballot + popcount
//   k_octree                  DistributeOctTree :542-766 -- one workgroup per (image, level); the
//                             list/push_front/erase order of the reference is reproduced with
//                             parallel passes (block scans + a bitonic sort of the refinement set)
//   k_blur                    GaussianBlur 7x7 :1083-1084 of every level, bit-exact fixed point
//   k_describe                IC_Angle :75-102 + computeOrbDescriptor :105-151 + rescale
//                             :1093-1099 -- one wavefront per keypoint; the 256 tests land as 4
//                             wave ballots (= 32 bytes)
// Data layout in HBM per image: pyramid levels 0..L-1 packed, rows padded to a 64-byte pitch with
// REFLECT_101 columns on both sides; the blurred pyramid in the same layout; FAST candidate slots
// per cell (u32 x | y<<12 | score<<24, cell order); octree key scratch for levels too large for
// LDS; per-level survivor keys; outputs orbfe_keypoint[cap] + 32-byte descriptors[cap] + count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_debug.h"
#include "orb_pattern31.inc"
#include "orbfe_device.h"
#include "orbfe_internal.h"
#include "orbfe_ktimer.h"

// ---------------------------------------------------------------------------------------------
// errors
static thread_local std::string g_last_error;
int orbfe_set_error(int code, const char* msg) {
  g_last_error = msg ? msg : "";
  return code;
}
int orbfe_set_hip_error(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return ORBFE_ERR_HIP;
}
extern "C" const char* orbfe_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* orbfe_version(void) { return "orbfe 0.1 gfx950"; }

// ---------------------------------------------------------------------------------------------
// geometry tables (host-computed, uploaded once per image shape)
struct LevelDesc {
  int w, h, pitch;
  int blur_h;                // k_blur: row bands per wavefront of the narrow last column strip (0: none)
  long long pyr_off;     // byte offset of column 0, row 0 of this level in one image's block
  int cell_begin, ncells;
  int cand_begin, cand_cap;  // candidate slots of this level inside one image's candidate block
  int budget;                // mnFeaturesPerLevel[l]
  int nini;                  // DistributeOctTree initial nodes (:546)
  float hx;                  // (:548)
  int rel_w, rel_h;          // maxBorderX - minBorderX, maxBorderY - minBorderY
  int key_begin, key_cap;    // octree output slots of this level inside one image's key block
  float scale;               // mvScaleFactor[l]
  int size;                  // scaledPatchSize (:840)
  int tab_x, tab_y;          // resize table offsets (l >= 1)
  int xmax, simd_end;        // resize: first column using the clamped path / end of SIMD columns
  int tile_begin, tiles_x;   // k_blur tiles of this level; full-width (BS_W) column strips
  int rgrp_begin, rwin_ok;   // k_resize 4-column group tables; 1 when every group's taps fit 8 bytes
  int ini_thr[8];            // smallest x with (int)(x / hx) >= b, b = 1..7 (initial node of key x)
};

struct CellDesc {
  int16_t level, x0, y0, rw, rh, ox, oy, pad;
  int32_t slot, cap;
  int32_t pyr_off, pitch;  // the level's (LevelDesc): k_fast's ROI address needs no second descriptor load
};

struct ExtractArgs {
  const LevelDesc* levels;
  const CellDesc* cells;
  const int2* xtab;
  const int2* ytab;
  const int4* ywin;  // k_resize_win: per output row the clamped source rows as dword offsets, betas
  int nlevels, ncells, n_images, total_key_slots, blur_strips;
  const uint8_t* img0;
  long long img_stride;
  int img_pitch, pad1;
  uint8_t* pyr;
  uint8_t* blur;  // blurred levels, same layout as pyr
  long long pyr_stride;
  uint32_t* cand;
  long long cand_stride;
  int32_t* cellcnt;
  uint32_t* keys_a;
  uint32_t* keys_b;
  long long keyscr_stride;
  uint32_t* lvlkeys;
  long long lvlkey_stride;
  int32_t* lvlcnt;
  orbfe_keypoint* out_kps;
  uint8_t* out_desc;
  int32_t* out_counts;
  int out_cap;
  int ini_th, min_th;
  int roi_w_max, roi_h_max;
  int node_cap, sort_cap, scan_cap, key_lds_cap;
  int oct_small;          // k_octree: nodes of <= oct_small keys split by one thread, larger by a wavefront
  const uint4* rgrp;      // k_resize: per 4-column group {sel[4]}, {alpha[4]} (2 x uint4)
  const int* rgx0;        // k_resize: first source column of each group
  int umax[16];
  AtanConsts atan;
  float factor_pi;
};

__constant__ int8_t c_pattern[1024];


__device__ __forceinline__ const uint8_t* level_ptr(const ExtractArgs& a, const LevelDesc& ld,
                                                    int img, int l, int& pitch) {
  (void)l;  // every level, the copied input included, lives in the pyramid block
  pitch = ld.pitch;
  return a.pyr + (long long)img * a.pyr_stride + ld.pyr_off;
}

__device__ __forceinline__ int sat16(int v) { return min(max(v, -32768), 32767); }

// Four output pixels x..x+3 of one row of level `ld` (resize INTER_LINEAR, ORBextractor.cc:1118):
// source rows r0/r1 (level width sw), OpenCV's fixed-point horizontal pass and, for x below
// simd_end, the SIMD128 vertical rounding (VResizeLinearVec_32s8u), else FixedPtCast<int,uchar,22>.
struct Taps4 {
  int p00[4], p01[4], p10[4], p11[4];
};

// the 16 source bytes of 4 output pixels (independent loads, all in flight together)
__device__ __forceinline__ Taps4 gather4(const uint8_t* r0, const uint8_t* r1, const int2* xt, int sw) {
  Taps4 t;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int sx = xt[k].x, sx1 = min(sx + 1, sw - 1);  // (sx1 only used below xmax, where sx+1 < sw)
    t.p00[k] = r0[sx];
    t.p01[k] = r0[sx1];
    t.p10[k] = r1[sx];
    t.p11[k] = r1[sx1];
  }
  return t;
}

__device__ __forceinline__ uint32_t combine4(const Taps4& t, const int2* xt, int x, const LevelDesc& ld,
                                             int b0, int b1) {
  const int *p00 = t.p00, *p01 = t.p01, *p10 = t.p10, *p11 = t.p11;
  uint32_t packed = 0;
  if (x + 3 < ld.xmax && x + 3 < ld.simd_end) {
    // interior (the common case): both taps in range and the SIMD128 rounding; the saturations of
    // VResizeLinearVec_32s8u never bind here (h <= 255 * 2048, betas in [0, 2048])
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int a0 = (int)(short)(xt[k].y & 0xffff), a1 = (int)(short)((unsigned)xt[k].y >> 16);
      const int h0 = p00[k] * a0 + p01[k] * a1, h1 = p10[k] * a0 + p11[k] * a1;
      const int m0 = ((h0 >> 4) * b0) >> 16, m1 = ((h1 >> 4) * b1) >> 16;
      packed |= (uint32_t)((m0 + m1 + 2) >> 2) << (8 * k);
    }
    return packed;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int xx = x + k;
    const int a0 = (int)(short)(xt[k].y & 0xffff), a1 = (int)(short)((unsigned)xt[k].y >> 16);
    int h0, h1;
    if (xx < ld.xmax) {
      h0 = p00[k] * a0 + p01[k] * a1;
      h1 = p10[k] * a0 + p11[k] * a1;
    } else {
      h0 = p00[k] * 2048;
      h1 = p10[k] * 2048;
    }
    int v;
    if (xx < ld.simd_end) {  // VResizeLinearVec_32s8u (v_mul_hi, saturating adds, rshr_pack_u<2>)
      const int m0 = (sat16(h0 >> 4) * b0) >> 16, m1 = (sat16(h1 >> 4) * b1) >> 16;
      v = sat16(sat16(m0 + m1) + 2) >> 2;
    } else {  // FixedPtCast<int, uchar, 22>
      v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    }
    packed |= (uint32_t)min(max(v, 0), 255) << (8 * k);
  }
  return packed;
}

template <typename XT>
__device__ __forceinline__ uint32_t resize4(const uint8_t* r0, const uint8_t* r1, XT xtab, int x,
                                            const LevelDesc& ld, int sw, int b0, int b1) {
  int2 xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) xt[k] = xtab[min(x + k, ld.w - 1)];
  return combine4(gather4(r0, r1, xt, sw), xt, x, ld, b0, b1);
}

// Store 4 bytes of a pyramid row at column x (n = valid bytes) plus the REFLECT_101 padding
// columns -3..-1 and w..w+2 that k_blur reads.
__device__ __forceinline__ void store_row4(uint8_t* row, int x, int w, uint32_t packed) {
  if (x >= 4 && x + 8 <= w) {  // interior: no padding column is a reflection of these 4
    *reinterpret_cast<uint32_t*>(row + x) = packed;
    return;
  }
  const int n = min(4, w - x);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int xx = x + k;
    const uint8_t b = (uint8_t)(packed >> (8 * k));
    if (k < n) {
      if (xx >= 1 && xx <= 3) row[-xx] = b;
      if (xx >= w - 4 && xx <= w - 2) row[2 * w - 2 - xx] = b;
    }
  }
  if (n == 4) *reinterpret_cast<uint32_t*>(row + x) = packed;
  else
    for (int k = 0; k < n; k++) row[x + k] = (uint8_t)(packed >> (8 * k));  // keep the padding bytes
}

// ---------------------------------------------------------------------------------------------
// k_resize: level l from level l-1 (ComputePyramid, ORBextractor.cc:1105-1135), one launch per
// level -- the fallback of k_resize_win for scale factors whose taps do not fit an 8-byte window.
#define RESIZE_ROWS 8  // output rows per thread (the column taps are loaded once)
__global__ __launch_bounds__(256) void k_resize(ExtractArgs a, int l) {
  const LevelDesc ld = a.levels[l];
  const int x = (blockIdx.x * 64 + threadIdx.x) * 4;  // 4 output pixels per thread
  const int ybeg = (blockIdx.y * 4 + threadIdx.y) * RESIZE_ROWS;
  const int img = blockIdx.z;
  if (x >= ld.w || ybeg >= ld.h) return;
  const int yend = min(ybeg + RESIZE_ROWS, ld.h);
  const LevelDesc ls = a.levels[l - 1];
  int spitch;
  const uint8_t* src = level_ptr(a, ls, img, l - 1, spitch);
  int2 xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) xt[k] = a.xtab[ld.tab_x + min(x + k, ld.w - 1)];
  const int2* ytab = a.ytab + ld.tab_y;
  uint8_t* out = a.pyr + (long long)img * a.pyr_stride + ld.pyr_off;
  for (int y = ybeg; y < yend; y += 2) {
    const bool two = y + 1 < yend;
    const int2 ya = ytab[y], yb = ytab[two ? y + 1 : y];
    const uint8_t* ra0 = src + (long long)min(max(ya.x, 0), ls.h - 1) * spitch;
    const uint8_t* ra1 = src + (long long)min(max(ya.x + 1, 0), ls.h - 1) * spitch;
    const uint8_t* rb0 = src + (long long)min(max(yb.x, 0), ls.h - 1) * spitch;
    const uint8_t* rb1 = src + (long long)min(max(yb.x + 1, 0), ls.h - 1) * spitch;
    const Taps4 ta = gather4(ra0, ra1, xt, ls.w);
    const Taps4 tb = gather4(rb0, rb1, xt, ls.w);
    const uint32_t pa = combine4(ta, xt, x, ld, (int)(short)(ya.y & 0xffff), (int)(short)((unsigned)ya.y >> 16));
    store_row4(out + (long long)y * ld.pitch, x, ld.w, pa);
    if (two) {
      const uint32_t pb = combine4(tb, xt, x, ld, (int)(short)(yb.y & 0xffff), (int)(short)((unsigned)yb.y >> 16));
      store_row4(out + (long long)(y + 1) * ld.pitch, x, ld.w, pb);
    }
  }
}

// k_resize_win: the same level step with the taps of 4 output columns gathered from one 8-byte
// source window per row: 3 aligned dword loads + 2 v_alignbyte per source row, then per pixel one
// v_perm (the two taps as u16 halves) and one v_dot2_u32_u16 with the packed alphas. Two output
// rows per thread (4 source rows, 12 loads in flight). Used when every group's taps span <= 8
// bytes (LevelDesc::rwin_ok; scale factors up to ~1.6).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2_u16(uint32_t a, uint32_t b) {
  return (int)__builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), 0u, false);
}
// a.lo * b.lo + a.hi * b.hi + c (v_dot2_u32_u16 with its accumulator operand)
__device__ __forceinline__ uint32_t dot2_acc(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c, false);
}

// bits 32..47 of the 48-bit product of two 24-bit values (v_mul_hi_u32_u24, full rate)
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// One output row of the 4-column group at x of level ld from the 8-byte windows (W0, W1) of its
// two source rows. Horizontal taps: one v_perm + one v_dot2_u32_u16 per pixel and source row with
// the alphas premultiplied by 16 (a16 <= 32768 still fits a u16 half), so H = 16 h and
// H & ~0xff = (h >> 4) << 8. OpenCV's SIMD128 vertical rounding (VResizeLinearVec_32s8u, whose
// saturations never bind here) ((h >> 4) * b) >> 16 is then one full-rate v_mul_hi_u32_u24 of
// (H & ~0xff) and b << 8 (both < 2^24; bits 32..47 of the product). Columns at or past simd_end
// take FixedPtCast<int, uchar, 22> on h = H >> 4 (TAIL: groups reaching simd_end).
template <bool TAIL>
__device__ __forceinline__ uint32_t resize_win_row(const uint32_t W0r0, const uint32_t W1r0, const uint32_t W0r1,
                                                   const uint32_t W1r1, const uint4 sel, const uint4 alp16,
                                                   int x, const LevelDesc& ld, int2 yt) {
  const uint32_t b0 = yt.y & 0xffffu, b1 = (uint32_t)yt.y >> 16;
  const uint32_t sels[4] = {sel.x, sel.y, sel.z, sel.w}, alps[4] = {alp16.x, alp16.y, alp16.z, alp16.w};
  uint32_t H0[4], H1[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    H0[k] = (uint32_t)dot2_u16(__builtin_amdgcn_perm(W1r0, W0r0, sels[k]), alps[k]);
    H1[k] = (uint32_t)dot2_u16(__builtin_amdgcn_perm(W1r1, W0r1, sels[k]), alps[k]);
  }
  uint32_t packed = 0;
  if constexpr (!TAIL) {  // every column below simd_end: the SIMD128 rounding only
    const uint32_t B0 = b0 << 8, B1 = b1 << 8;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t m0 = mulhi_u24(H0[k] & 0xffff00u, B0);
      const uint32_t m1 = mulhi_u24(H1[k] & 0xffff00u, B1);
      packed |= ((m0 + m1 + 2u) >> 2) << (8 * k);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int h0 = (int)(H0[k] >> 4), h1 = (int)(H1[k] >> 4);
      int v;
      if (x + k < ld.simd_end) {
        v = ((((h0 >> 4) * (int)b0) >> 16) + (((h1 >> 4) * (int)b1) >> 16) + 2) >> 2;
      } else {
        v = min(max((h0 * (int)b0 + h1 * (int)b1 + (1 << 21)) >> 22, 0), 255);
      }
      packed |= (uint32_t)v << (8 * k);
    }
  }
  return packed;
}

// Items (4-column group, row pair) of the level are numbered row-major and dealt to the threads
// linearly, so only the last wave of an image's grid has idle lanes (a 2-D grid of 256-column
// blocks left up to a third of the lanes idle on the right edge of every row band). One row pair
// per thread (2 and 4 pairs with every source row in flight measured slower).
__global__ __launch_bounds__(256) void k_resize_win(ExtractArgs a, int l, int G, uint32_t gmagic) {
  const LevelDesc ld = a.levels[l];
  const int item = blockIdx.x * 256 + threadIdx.x, img = blockIdx.y;
  const int pr = gmagic ? (int)__umulhi((uint32_t)item, gmagic) : item;  // item / G
  const int g = item - pr * G, x = 4 * g;
  const int y0 = 2 * pr;
  if (y0 >= ld.h) return;
  const LevelDesc ls = a.levels[l - 1];
  // the source level as dwords from a wave-uniform base; per-lane offsets are 32-bit unsigned
  // (row offsets precomputed and clamped on the host: LevelDesc rows are 4-byte aligned)
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.pyr + (long long)img * a.pyr_stride + ls.pyr_off);
  const uint32_t gi = (uint32_t)(ld.rgrp_begin + g);
  const uint32_t sx0 = (uint32_t)a.rgx0[gi];
  const uint4 sel = a.rgrp[2 * gi], alp16 = a.rgrp[2 * gi + 1];
  const uint32_t cx = sx0 >> 2;
  const int4 ya = a.ywin[(uint32_t)(ld.tab_y + y0)], yb = a.ywin[(uint32_t)(ld.tab_y + min(y0 + 1, ld.h - 1))];
  const uint32_t rows[4] = {(uint32_t)ya.x + cx, (uint32_t)ya.y + cx, (uint32_t)yb.x + cx, (uint32_t)yb.y + cx};
  // raw buffer loads from the wave-uniform base: 32-bit byte offsets, no per-lane 64-bit math
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), 0, 0x7fffffff, 0x00020000);
  uint32_t wv[4][3];
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int k = 0; k < 3; k++) wv[r][k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * rows[r]) + 4 * k, 0, 0);
  }
  const int sh = (int)(sx0 & 3u);
  uint32_t W0[4], W1[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    W0[r] = __builtin_amdgcn_alignbyte(wv[r][1], wv[r][0], sh);
    W1[r] = __builtin_amdgcn_alignbyte(wv[r][2], wv[r][1], sh);
  }
  uint8_t* out = a.pyr + (long long)img * a.pyr_stride + ld.pyr_off;
  const int2 ba = make_int2(0, ya.z), bb = make_int2(0, yb.z);
  uint32_t pa, pb;
  if (x + 4 <= ld.simd_end) {  // every column on the SIMD128 rounding (all but a row's tail)
    pa = resize_win_row<false>(W0[0], W1[0], W0[1], W1[1], sel, alp16, x, ld, ba);
    pb = resize_win_row<false>(W0[2], W1[2], W0[3], W1[3], sel, alp16, x, ld, bb);
  } else {
    pa = resize_win_row<true>(W0[0], W1[0], W0[1], W1[1], sel, alp16, x, ld, ba);
    pb = resize_win_row<true>(W0[2], W1[2], W0[3], W1[3], sel, alp16, x, ld, bb);
  }
  store_row4(out + __umul24((uint32_t)y0, (uint32_t)ld.pitch), x, ld.w, pa);
  if (y0 + 1 < ld.h) store_row4(out + __umul24((uint32_t)(y0 + 1), (uint32_t)ld.pitch), x, ld.w, pb);
}

// k_pyramid: levels 1..L-1 of ComputePyramid (ORBextractor.cc:1105-1135) in ONE launch, the chain
// of dependent per-level resizes kept inside each workgroup. The image is cut into tx x ty tiles
// per level (PyrTileLevel, host-planned by pyramid_plan); a workgroup owns one tile of every level
// and computes, level after level, its owned 4-column groups and rows plus the halo the next
// level's computed region reads (the dependency cone, at most a few rows / groups per side), with
// level l-1 held in LDS while level l is built (two LDS buffers, one barrier per level); level 1
// reads level 0 from the pyramid block. Owned pixels (and their REFLECT_101 padding columns) go to
// the pyramid block; halo pixels are recomputed by the neighbouring tiles from the same source
// bytes with the same arithmetic as k_resize_win, so the result is the per-level chain's byte for
// byte. Replaces L-1 launches (each a latency-bound grid that leaves most CUs idle, plus a kernel
// boundary) by one, and level l-1's bytes are read from LDS instead of L2 / HBM.
struct PyrTileLevel {
  int16_t ng_a, ng_b, ny_a, ny_b;  // computed groups [ng_a, ng_b) and rows [ny_a, ny_b)
  int16_t og_a, og_b, oy_a, oy_b;  // owned (stored): a subset of the computed region
  uint32_t gmagic;                 // item / (4 (ng_b - ng_a)) as __umulhi(item, gmagic)
  int32_t tab_off;                 // this level's staged tables in LDS (dwords; entries 9 per group, 2 per row)
};
constexpr int PYR_MAX_LEVELS = 32;
constexpr int PYR_LV_DW = 8;  // staged LevelDesc fields per level

// The tables one tile reads (per computed 4-column group its first source column and byte
// selectors / alphas, per computed row the source row and betas) and the level fields are staged in
// LDS first, all loads in flight together, so the level loop touches global memory only for level
// 0's bytes and the owned stores (one dependent table fetch per level measured ~3 us per level).
// A workgroup barrier that orders LDS only: __syncthreads() also waits for every outstanding
// global store (s_waitcnt vmcnt(0)), ~2-3 us per level here for pyramid bytes no workgroup of this
// launch reads back.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int PYR_NT = 1024;  // k_pyramid's workgroup
__global__ __launch_bounds__(PYR_NT) void k_pyramid(ExtractArgs a, const PyrTileLevel* __restrict__ tiles,
                                                 int half_dw, int dbg) {
#ifdef ORBFE_PYR_CLOCKS  // phase clocks of two workgroups (printf; a timing build only)
  unsigned long long tclk[40];
  int nclk = 0;
#define PYR_CLK() if (dbg) tclk[nclk++] = __builtin_amdgcn_s_memrealtime();
#else
#define PYR_CLK()
#endif
  PYR_CLK();
  extern __shared__ __attribute__((aligned(16))) uint32_t s_pyr[];
  __shared__ PyrTileLevel s_t[PYR_MAX_LEVELS];
  __shared__ int s_lv[PYR_MAX_LEVELS][PYR_LV_DW];  // w, h, pitch, pyr_off, simd_end, rgrp_begin, tab_y
  const int L = a.nlevels, tid = threadIdx.x;
  const int img = blockIdx.y;
  {
    const PyrTileLevel* T = tiles + (size_t)blockIdx.x * L;
    const int nT = L * (int)(sizeof(PyrTileLevel) / 4);
    if (tid < nT) reinterpret_cast<int*>(s_t)[tid] = reinterpret_cast<const int*>(T)[tid];
    const int u = tid - 128;
    if (u >= 0 && u < L * 7) {
      const int l = u / 7, f = u - 7 * l;
      const LevelDesc* d = a.levels + l;
      const int v = f == 0 ? d->w : f == 1 ? d->h : f == 2 ? d->pitch : f == 3 ? (int)d->pyr_off
                  : f == 4 ? d->simd_end : f == 5 ? d->rgrp_begin : d->tab_y;
      s_lv[l][f] = v;
    }
  }
  __syncthreads();
  PYR_CLK();
  uint32_t* s_tab = s_pyr + 2 * half_dw;
  {
    const int last = L - 1;
    const int total = s_t[last].tab_off + 9 * (s_t[last].ng_b - s_t[last].ng_a) + 2 * (s_t[last].ny_b - s_t[last].ny_a);
    const uint32_t* rg = reinterpret_cast<const uint32_t*>(a.rgrp);
    const uint32_t* yt = reinterpret_cast<const uint32_t*>(a.ytab);
    for (int e0 = tid; e0 < total; e0 += 4 * PYR_NT) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int e = e0 + PYR_NT * k;
        v[k] = 0;
        if (e < total) {
          int l = 1;
          while (l < last && e >= s_t[l + 1].tab_off) l++;
          const PyrTileLevel& t = s_t[l];
          const int j = e - t.tab_off, G9 = 9 * (t.ng_b - t.ng_a);
          if (j < G9) {
            const int g = j / 9, w = j - 9 * g;
            const uint32_t gi = (uint32_t)(s_lv[l][5] + t.ng_a + g);
            v[k] = w == 0 ? (uint32_t)a.rgx0[gi] : rg[8 * gi + (w - 1)];
          } else {
            const int r = j - G9;
            v[k] = yt[2 * (s_lv[l][6] + t.ny_a + (r >> 1)) + (r & 1)];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (e0 + PYR_NT * k < total) s_tab[e0 + PYR_NT * k] = v[k];
    }
  }
  __syncthreads();
  PYR_CLK();
  // (uniform values read from LDS go through readfirstlane: scalar registers, and the level-0
  // buffer descriptor stays scalar instead of a per-load waterfall loop)
  auto uni = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
  uint8_t* base = a.pyr + (long long)img * a.pyr_stride;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + uni(s_lv[0][3]), 0, 0x7fffffff, 0x00020000);
  const uint32_t pdw0 = (uint32_t)uni(s_lv[0][2]) >> 2;
  for (int l = 1; l < L; l++) {
    PyrTileLevel t = s_t[l], tp = s_t[l - 1];
    t.ng_a = (int16_t)uni(t.ng_a), t.ng_b = (int16_t)uni(t.ng_b), t.ny_a = (int16_t)uni(t.ny_a);
    t.ny_b = (int16_t)uni(t.ny_b), t.og_a = (int16_t)uni(t.og_a), t.og_b = (int16_t)uni(t.og_b);
    t.oy_a = (int16_t)uni(t.oy_a), t.oy_b = (int16_t)uni(t.oy_b), t.gmagic = (uint32_t)uni((int)t.gmagic);
    t.tab_off = uni(t.tab_off);
    tp.ng_a = (int16_t)uni(tp.ng_a), tp.ng_b = (int16_t)uni(tp.ng_b), tp.ny_a = (int16_t)uni(tp.ny_a);
    const int w = uni(s_lv[l][0]), pitch = uni(s_lv[l][2]), simd_end = uni(s_lv[l][4]), hs = uni(s_lv[l - 1][1]);
    const int ng = t.ng_b - t.ng_a, nc = 4 * ng;
    const int items = ng > 0 ? nc * ((t.ny_b - t.ny_a + 1) >> 1) : 0;
    uint8_t* dst = reinterpret_cast<uint8_t*>(s_pyr + (l & 1) * half_dw);
    const uint32_t* srcl = s_pyr + ((l - 1) & 1) * half_dw;
    const uint32_t* tg = s_tab + t.tab_off;
    const uint32_t* ty = tg + 9 * ng;
    const int dpitch = 4 * (ng + 3), spitch = tp.ng_b - tp.ng_a + 3;
    const bool keep = l + 1 < L;
    uint8_t* out = base + uni(s_lv[l][3]);
    // one output pixel (column x, rows y0 and y0 + 1) per thread: the group's window and tables
    // are read by its 4 lanes (LDS broadcast), each lane its own selector / alpha pair
    for (int item = tid; item < items; item += PYR_NT) {
      const int pr = t.gmagic ? (int)__umulhi((uint32_t)item, t.gmagic) : item;
      const int xo = item - pr * nc, gl = xo >> 2, k = xo & 3;
      const int g = t.ng_a + gl, x = 4 * t.ng_a + xo;
      const int y0 = t.ny_a + 2 * pr;
      const bool two = y0 + 1 < t.ny_b;
      const uint32_t* q = tg + 9 * gl;
      const uint32_t sx0 = q[0], sel = q[1 + k], alp16 = q[5 + k];
      const int ra = 2 * (y0 - t.ny_a), rb = two ? ra + 2 : ra;
      const int2 ya = make_int2((int)ty[ra], (int)ty[ra + 1]), yb = make_int2((int)ty[rb], (int)ty[rb + 1]);
      const int rr[4] = {min(max(ya.x, 0), hs - 1), min(max(ya.x + 1, 0), hs - 1), min(max(yb.x, 0), hs - 1),
                         min(max(yb.x + 1, 0), hs - 1)};
      uint32_t wv[4][3];
      if (l == 1) {  // level 0 from the pyramid block: 3 aligned dwords per source row
        const uint32_t cx = sx0 >> 2;
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
          for (int kk = 0; kk < 3; kk++)
            wv[r][kk] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * ((uint32_t)rr[r] * pdw0 + cx)) + 4 * kk, 0, 0);
        }
      } else {  // level l-1 from this tile's LDS copy
        const int c = (int)(sx0 >> 2) - tp.ng_a;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint32_t* p = srcl + (rr[r] - tp.ny_a) * spitch + c;
#pragma unroll
          for (int kk = 0; kk < 3; kk++) wv[r][kk] = p[kk];
        }
      }
      const int sh = (int)(sx0 & 3u);
      uint32_t H[4];  // 16 h of the 4 source rows (resize_win_row's horizontal pass, one column)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t W0 = __builtin_amdgcn_alignbyte(wv[r][1], wv[r][0], sh);
        const uint32_t W1 = __builtin_amdgcn_alignbyte(wv[r][2], wv[r][1], sh);
        H[r] = (uint32_t)dot2_u16(__builtin_amdgcn_perm(W1, W0, sel), alp16);
      }
      uint32_t va, vb;
      const uint32_t ba0 = (uint32_t)ya.y & 0xffffu, ba1 = (uint32_t)ya.y >> 16;
      const uint32_t bb0 = (uint32_t)yb.y & 0xffffu, bb1 = (uint32_t)yb.y >> 16;
      if (x < simd_end) {  // OpenCV's SIMD128 vertical rounding (resize_win_row)
        va = (mulhi_u24(H[0] & 0xffff00u, ba0 << 8) + mulhi_u24(H[1] & 0xffff00u, ba1 << 8) + 2u) >> 2;
        vb = (mulhi_u24(H[2] & 0xffff00u, bb0 << 8) + mulhi_u24(H[3] & 0xffff00u, bb1 << 8) + 2u) >> 2;
      } else {  // FixedPtCast<int, uchar, 22>
        const int h0 = (int)(H[0] >> 4), h1 = (int)(H[1] >> 4), h2 = (int)(H[2] >> 4), h3 = (int)(H[3] >> 4);
        va = (uint32_t)min(max((h0 * (int)ba0 + h1 * (int)ba1 + (1 << 21)) >> 22, 0), 255);
        vb = (uint32_t)min(max((h2 * (int)bb0 + h3 * (int)bb1 + (1 << 21)) >> 22, 0), 255);
      }
      if (keep) {
        uint8_t* d = dst + (y0 - t.ny_a) * dpitch + xo;
        d[0] = (uint8_t)va;
        if (two) d[dpitch] = (uint8_t)vb;
      }
      if (g >= t.og_a && g < t.og_b && x < w) {  // owned: the byte and its REFLECT_101 copies (store_row4)
        const int xr = x >= 1 && x <= 3 ? -x : x >= w - 4 && x <= w - 2 ? 2 * w - 2 - x : INT_MIN;
        if (y0 >= t.oy_a && y0 < t.oy_b) {
          uint8_t* row = out + __umul24((uint32_t)y0, (uint32_t)pitch);
          row[x] = (uint8_t)va;
          if (xr != INT_MIN) row[xr] = (uint8_t)va;
        }
        if (two && y0 + 1 >= t.oy_a && y0 + 1 < t.oy_b) {
          uint8_t* row = out + __umul24((uint32_t)(y0 + 1), (uint32_t)pitch);
          row[x] = (uint8_t)vb;
          if (xr != INT_MIN) row[xr] = (uint8_t)vb;
        }
      }
    }
    lds_barrier();  // the next level reads this one's LDS copy; the pyramid stores stay in flight
    PYR_CLK();
  }
#ifdef ORBFE_PYR_CLOCKS
  if (dbg && threadIdx.x == 0 && blockIdx.x == gridDim.x / 2 && blockIdx.y == 0) {
    printf("pyr blk %d:", blockIdx.x);
    for (int i = 1; i < nclk; i++) printf(" %d", (int)(tclk[i] - tclk[i - 1]));
    printf("\n");
  }
#endif
  (void)dbg;
}


// k_copy_l0: level 0 from a host staging buffer the caller-side code already laid out like the
// pyramid block (rows `pitch` apart, the REFLECT_101 columns filled on the host): one straight copy
// of pitch x h bytes, 16-byte loads, four per thread in flight -- the zero-copy path of the small
// host calls, where the loads cross PCIe and k_copy0's row-by-row dword loads of an unaligned row
// ran at ~23 GB/s.
__global__ __launch_bounds__(256) void k_copy_l0(ExtractArgs a) {
  const LevelDesc ld = a.levels[0];
  const int img = blockIdx.y;
  const int n16 = (ld.pitch * ld.h) >> 4;
  const uint4* src = reinterpret_cast<const uint4*>(a.img0 + (long long)img * a.img_stride);
  uint4* dst = reinterpret_cast<uint4*>(a.pyr + (long long)img * a.pyr_stride + ld.pyr_off - 4);
  const int i0 = blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + 256 * k;
    if (i < n16) v[k] = src[i];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + 256 * k;
    if (i < n16) dst[i] = v[k];
  }
}

// k_copy0: the input image into level 0 of the pyramid block (64-byte aligned rows, REFLECT_101
// padding columns).
__global__ __launch_bounds__(256) void k_copy0(ExtractArgs a) {
  // One wavefront per row. The caller's row (any pitch, any byte alignment) comes in as coalesced
  // aligned dwords into LDS (byte loads only for a last dword that would run past the row); the
  // padded pyramid row goes out as 16-byte stores of its physical chunks (bytes past column w+2
  // and column -4 are don't-care padding), then six lanes patch the REFLECT_101 columns -3..-1
  // and w..w+2. (The previous mapping, 16 columns per thread with 5 dword loads and per-dword
  // stores, took 57-65 us per 64 KITTI images alone.)
  extern __shared__ __attribute__((aligned(16))) uint32_t s_rows[];
  const LevelDesc ld = a.levels[0];
  const int w = ld.w, lane = lane_id(), wv = wave_id();
  const int y = blockIdx.x * 4 + wv, img = blockIdx.y;
  if (y >= ld.h) return;
  const int rd = (ld.pitch >> 2) + 4;  // LDS dwords per wave: one before the row, the row, slack
  uint32_t* s = s_rows + wv * rd + 1;
  const uint8_t* src = a.img0 + (long long)img * a.img_stride + (long long)y * a.img_pitch;
  const int sh = (int)(reinterpret_cast<uintptr_t>(src) & 3);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(src - sh);
  const int nd = (sh + w + 3) >> 2;  // dwords holding columns 0..w-1 (and up to 3 bytes before)
  const int nfull = (sh + w) >> 2;   // dwords wholly inside the row
  // the row's whole dwords: up to 8 per lane issued before any is stored (one memory latency per
  // row instead of one per 64 dwords; rows up to 2048 dwords), a strided loop past that
  constexpr int CU = 8;
  uint32_t v8[CU];
#pragma unroll
  for (int k = 0; k < CU; k++) {
    const int i = lane + 64 * k;
    v8[k] = i < nfull ? p[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < CU; k++) {
    const int i = lane + 64 * k;
    if (i < nfull) s[i] = v8[k];
  }
  for (int i = lane + 64 * CU; i < nfull; i += 64) s[i] = p[i];
  if (lane == 0 && nfull < nd) {  // the row's last dword: only its bytes inside the row
    uint32_t v = 0;
    for (int j = 0; j < 4; j++)
      if (4 * nfull + j >= sh && 4 * nfull + j < sh + w) v |= (uint32_t)src[4 * nfull + j - sh] << (8 * j);
    s[nfull] = v;
  }
  wave_sync();
  uint8_t* row = a.pyr + (long long)img * a.pyr_stride + ld.pyr_off - 4 + (long long)y * ld.pitch;
  const int nchunks = ld.pitch >> 4;  // physical bytes 0..pitch-1 = columns -4 .. pitch-5
  for (int P = lane; P < nchunks; P += 64) {
    const int b = sh + 16 * P - 4;  // LDS byte of the chunk's first column (>= -4)
    const int r = b & 3;
    const uint32_t* q = s + (b >> 2);  // arithmetic shift: b = -4..-1 -> s[-1]
    uint32_t w5[5];
#pragma unroll
    for (int k = 0; k < 5; k++) w5[k] = q[k];
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(w5[1], w5[0], r);
    o.y = __builtin_amdgcn_alignbyte(w5[2], w5[1], r);
    o.z = __builtin_amdgcn_alignbyte(w5[3], w5[2], r);
    o.w = __builtin_amdgcn_alignbyte(w5[4], w5[3], r);
    *reinterpret_cast<uint4*>(row + 16 * P) = o;
  }
  __builtin_amdgcn_s_waitcnt(0);  // the chunk stores before the patches of their padding bytes
  if (lane < 6) {
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(s) + sh;  // column c at sb[c]
    const int k = lane < 3 ? lane : lane - 3;
    const int col = lane < 3 ? -1 - k : w + k;                        // -1..-3, w..w+2
    const int from = lane < 3 ? min(1 + k, w - 1) : max(w - 2 - k, 0);  // REFLECT_101
    row[4 + col] = sb[from];
  }
}

// ---------------------------------------------------------------------------------------------
// FAST-9/16 helpers on an LDS tile with row stride `s` (OpenCV fast.cpp FAST_t<16>).
// Ring offsets (dx, dy) starting at (0, 3): makeOffsets(pixel, step, 16).
__device__ __forceinline__ int ring_off(int k, int s) {
  switch (k) {
    case 0: return 3 * s;
    case 1: return 1 + 3 * s;
    case 2: return 2 + 2 * s;
    case 3: return 3 + s;
    case 4: return 3;
    case 5: return 3 - s;
    case 6: return 2 - 2 * s;
    case 7: return 1 - 3 * s;
    case 8: return -3 * s;
    case 9: return -1 - 3 * s;
    case 10: return -2 - 2 * s;
    case 11: return -3 - s;
    case 12: return -3;
    case 13: return -3 + s;
    case 14: return -2 + 2 * s;
    default: return -1 + 3 * s;
  }
}

// Arc strength M = max(v - A, B - v) with A = min over the 16 arcs of 9 of the max ring value and
// B = max over arcs of the min ring value. The pixel is a FAST corner at threshold t iff
// M >= t+1, and then cornerScore<16> == M - 1. Returns 0 when the pixel is no corner at tlow.
// Callers run OpenCV's antipodal quick test first (it never rejects a corner).
__device__ __forceinline__ int arc_strength_nq(const uint8_t* p, int s, int tlow) {
  const int v = p[0];
  int x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = p[ring_off(k, s)];
  int mn2[16], mx2[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    mn2[k] = min(x[k], x[(k + 1) & 15]);
    mx2[k] = max(x[k], x[(k + 1) & 15]);
  }
  int mn4[16], mx4[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    mn4[k] = min(mn2[k], mn2[(k + 2) & 15]);
    mx4[k] = max(mx2[k], mx2[(k + 2) & 15]);
  }
  int B = 0, A = 255;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int mn9 = min(min(mn4[k], mn4[(k + 4) & 15]), x[(k + 8) & 15]);
    const int mx9 = max(max(mx4[k], mx4[(k + 4) & 15]), x[(k + 8) & 15]);
    B = max(B, mn9);
    A = min(A, mx9);
  }
  const int m = max(v - A, B - v);
  return m < tlow + 1 ? 0 : m;
}

// two u8 values in the 16-bit halves of a dword, and packed 16-bit add / subtract (v_pk_*_u16)
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(uint32_t lo, uint32_t hi) { return lo | (hi << 16); }
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, a) - __builtin_bit_cast(s16x2, b));
}
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}

// Arc strength of two pixels (pa -> low 16 bits, pb -> high 16 bits): M where M >= tlow + 1
// (exactly the FAST corners at tlow; see arc_strength_nq), else 0. The callers' prefilter has
// already dropped most non-corners, so OpenCV's full antipodal quick test is not repeated here.
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
typedef short i16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2v, a), __builtin_bit_cast(u16x2v, b)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2v, a), __builtin_bit_cast(u16x2v, b)));
}
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2v, a), __builtin_bit_cast(i16x2v, b)));
}
// 3-input packed min / max of byte pairs viewed as f16 (v_pk_minimum3_f16 / v_pk_maximum3_f16)
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f16_max3(uint32_t a, uint32_t b, uint32_t c) {
  const f16x2v r = __builtin_elementwise_maximum(
      __builtin_elementwise_maximum(__builtin_bit_cast(f16x2v, a), __builtin_bit_cast(f16x2v, b)),
      __builtin_bit_cast(f16x2v, c));
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t f16_min3(uint32_t a, uint32_t b, uint32_t c) {
  const f16x2v r = __builtin_elementwise_minimum(
      __builtin_elementwise_minimum(__builtin_bit_cast(f16x2v, a), __builtin_bit_cast(f16x2v, b)),
      __builtin_bit_cast(f16x2v, c));
  return __builtin_bit_cast(uint32_t, r);
}
// two LDS bytes into the halves of a dword (ds_read_u8 + ds_read_u8_d16_hi, no packing op)
__device__ __forceinline__ uint32_t lds_pair(const uint8_t* a, const uint8_t* b) {
  u16x2v v;
  v.x = a[0];
  v.y = b[0];
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint32_t arc_strength_pk(const uint8_t* pa, const uint8_t* pb, int s, int tlow) {
  const uint32_t c = lds_pair(pa, pb);
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = lds_pair(pa + ring_off(k, s), pb + ring_off(k, s));
  // A = min over the 16 arcs of 9 of the arc max, B = max over the arcs of the arc min, by the
  // gfx950 3-input packed f16 ops: a zero-extended byte is an f16 denormal whose order is the
  // integer order (f16 denormals are preserved, .amdhsa_float_denorm_mode_16_64 3), and min / max
  // return one of their inputs bit for bit, so A and B come out as the integer bytes.
  // Arc max over x[k..k+8] = max3 of three 3-wide maxima: 16 + 16 ops, then a min3 tree.
  uint32_t A, B;
  {
    uint32_t t3[16], t9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t3[k] = f16_max3(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) t9[k] = f16_max3(t3[k], t3[(k + 3) & 15], t3[(k + 6) & 15]);
    A = f16_min3(f16_min3(f16_min3(t9[0], t9[1], t9[2]), f16_min3(t9[3], t9[4], t9[5]), f16_min3(t9[6], t9[7], t9[8])),
                 f16_min3(t9[9], t9[10], t9[11]), f16_min3(f16_min3(t9[12], t9[13], t9[14]), t9[15], t9[15]));
  }
  {
    uint32_t t3[16], t9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t3[k] = f16_min3(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) t9[k] = f16_min3(t3[k], t3[(k + 3) & 15], t3[(k + 6) & 15]);
    B = f16_max3(f16_max3(f16_max3(t9[0], t9[1], t9[2]), f16_max3(t9[3], t9[4], t9[5]), f16_max3(t9[6], t9[7], t9[8])),
                 f16_max3(t9[9], t9[10], t9[11]), f16_max3(f16_max3(t9[12], t9[13], t9[14]), t9[15], t9[15]));
  }
  const uint32_t m = pk_max_i16(pk_sub16(c, A), pk_sub16(B, c));  // max(v - A, B - v), signed
  const int ma = (int)(short)(m & 0xffffu), mb = (int)(short)(m >> 16);
  const uint32_t ra = ma >= tlow + 1 ? (uint32_t)ma : 0u;
  const uint32_t rb = mb >= tlow + 1 ? (uint32_t)mb : 0u;
  return ra | (rb << 16);
}

// 2a on the constant-stride path: four horizontally adjacent detection pixels per lane from dword
// LDS reads. ROI row i holds global column x0a + j at byte j, so detection pixel (rr, cc) of a
// cell with xo = x0 & 3 sits at byte XO + 3 + cc of ROI row rr + 3; for cc = 4g the ten bytes
// XO + 4g .. XO + 4g + 9 (left ring point .. right ring point) lie in the four dwords from byte
// 4g, the up / down ring points in two dwords of rows rr and rr + 6. Bytes are split into the two
// packed-u16 pairs (0, 2) and (1, 3) by v_perm. Survivors go to `list` in row-major order (lane
// prefix of the per-lane counts from three ballots of the count bits).
__device__ __forceinline__ uint32_t pk_even(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c020c00u); }
__device__ __forceinline__ uint32_t pk_odd(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0c030c01u); }
__device__ __forceinline__ uint32_t quick2(uint32_t c, uint32_t u, uint32_t d, uint32_t l, uint32_t r,
                                           uint32_t T2) {
  const uint32_t X = pk_max_u16(pk_min_u16(u, d), pk_min_u16(l, r));
  const uint32_t Y = pk_min_u16(pk_max_u16(u, d), pk_max_u16(l, r));
  return pk_sub16(X, pk_sub16(c, T2)) | pk_sub16(pk_add16(c, T2), Y);
}
// ceil(2^20 / g): q * kMagic20[g] >> 20 == q / g for the item counts of one cell (a table, so that
// no division is hoisted into the kernel's prologue)
__constant__ uint32_t kMagic20[16] = {0u, 1048576u, 524288u, 349526u, 262144u, 209716u, 174763u, 149797u,
                                      131072u, 116509u, 104858u, 95326u, 87382u, 80660u, 74899u, 69906u};
template <int RSC, int XO>
__device__ __forceinline__ int fast_prefilter4(const uint8_t* roi, int dw, int dh, uint32_t T2, uint16_t* list) {
  static_assert(RSC % 4 == 0, "dword rows");
  constexpr int RD = RSC / 4;                         // row stride in dwords
  constexpr int OC = XO + 3, OR = XO + 6;             // centre / right byte offsets from 4g
  const int gw = (dw + 3) >> 2;  // <= 15 here (ROI <= 61 columns)
  const uint32_t gmagic = kMagic20[gw];
  const int items = gw * dh;
  int nlist = 0;
  for (int q0 = 0; q0 < items; q0 += 64) {
    const int q = q0 + lane_id();
    uint32_t m4 = 0;
    int px = 0;
    if (q < items) {
      const int rr = (int)(((uint32_t)q * gmagic) >> 20), g = q - rr * gw;
      px = (rr << 6) + 4 * g;  // list entry r << 6 | c (c < 64 on this path)
      const uint32_t* row = reinterpret_cast<const uint32_t*>(roi) + (rr + 3) * RD + g;
      const uint32_t* up = row - 3 * RD;
      const uint32_t* dn = row + 3 * RD;
      const uint32_t w0 = row[0], w1 = row[1], w2 = row[2];
      const uint32_t w3 = XO == 3 ? row[3] : 0u;
      const uint32_t l = XO == 0 ? w0 : __builtin_amdgcn_alignbyte(w1, w0, XO);
      uint32_t c, r, u, d;
      if constexpr (OC < 4) c = __builtin_amdgcn_alignbyte(w1, w0, OC);
      else if constexpr (OC == 4) c = w1;
      else c = __builtin_amdgcn_alignbyte(w2, w1, OC - 4);
      if constexpr (OR < 8) r = __builtin_amdgcn_alignbyte(w2, w1, OR - 4);
      else if constexpr (OR == 8) r = w2;
      else r = __builtin_amdgcn_alignbyte(w3, w2, OR - 8);
      if constexpr ((OC & 3) == 0) {
        u = up[OC >> 2];
        d = dn[OC >> 2];
      } else {
        u = __builtin_amdgcn_alignbyte(up[(OC >> 2) + 1], up[OC >> 2], OC & 3);
        d = __builtin_amdgcn_alignbyte(dn[(OC >> 2) + 1], dn[OC >> 2], OC & 3);
      }
      const uint32_t re = quick2(pk_even(c), pk_even(u), pk_even(d), pk_even(l), pk_even(r), T2);
      const uint32_t ro = quick2(pk_odd(c), pk_odd(u), pk_odd(d), pk_odd(l), pk_odd(r), T2);
      m4 = ((re >> 15) & 1u) | ((ro >> 14) & 2u) | ((re >> 29) & 4u) | ((ro >> 28) & 8u);
      const int nv = dw - 4 * g;
      if (nv < 4) m4 &= (1u << nv) - 1u;
    }
    const int n = __popc(m4);
    const uint64_t b0 = wave_ballot(n & 1), b1 = wave_ballot(n & 2), b2 = wave_ballot(n & 4);
    int pos = nlist + prefix_in_wave(b0) + 2 * prefix_in_wave(b1) + 4 * prefix_in_wave(b2);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (m4 & (1u << k)) list[pos] = (uint16_t)(px + k);
      pos += (m4 >> k) & 1u;
    }
    nlist += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  }
  return nlist;
}

// The same prefilter for cells whose detection rows fit 8 groups of 4 (dw <= 32: every full cell
// of the 30-pixel grid, whose cells are 30-32 pixels wide): lane = (row of 8, group), so a lane's
// group and its column mask are fixed for the whole cell and rows advance by a constant. The four
// sign bits land in bytes 0..3 of one dword by a single v_perm (bits 7, 15, 23, 31), masked by
// the precomputed column mask; a lane writes its survivors by a loop over its set bits.
template <int RSC, int XO>
__device__ __forceinline__ int fast_prefilter4_g8(const uint8_t* roi, int dw, int dh, uint32_t T2, uint16_t* list) {
  static_assert(RSC % 4 == 0, "dword rows");
  constexpr int RD = RSC / 4;
  constexpr int OC = XO + 3, OR = XO + 6;
  const int lane = lane_id(), g = lane & 7, rs = lane >> 3;
  const int nv = dw - 4 * g;
  const uint32_t vmask = nv >= 4 ? 0x80808080u : nv <= 0 ? 0u : (0x80808080u >> (8 * (4 - nv)));
  const uint32_t* row = reinterpret_cast<const uint32_t*>(roi) + (rs + 3) * RD + g;
  int nlist = 0;
  for (int r0 = 0; r0 < dh; r0 += 8, row += 8 * RD) {
    const int rr = r0 + rs;
    const uint32_t* up = row - 3 * RD;
    const uint32_t* dn = row + 3 * RD;
    const uint32_t w0 = row[0], w1 = row[1], w2 = row[2];
    const uint32_t w3 = XO == 3 ? row[3] : 0u;
    const uint32_t l = XO == 0 ? w0 : __builtin_amdgcn_alignbyte(w1, w0, XO);
    uint32_t c, r, u, d;
    if constexpr (OC < 4) c = __builtin_amdgcn_alignbyte(w1, w0, OC);
    else if constexpr (OC == 4) c = w1;
    else c = __builtin_amdgcn_alignbyte(w2, w1, OC - 4);
    if constexpr (OR < 8) r = __builtin_amdgcn_alignbyte(w2, w1, OR - 4);
    else if constexpr (OR == 8) r = w2;
    else r = __builtin_amdgcn_alignbyte(w3, w2, OR - 8);
    if constexpr ((OC & 3) == 0) {
      u = up[OC >> 2];
      d = dn[OC >> 2];
    } else {
      u = __builtin_amdgcn_alignbyte(up[(OC >> 2) + 1], up[OC >> 2], OC & 3);
      d = __builtin_amdgcn_alignbyte(dn[(OC >> 2) + 1], dn[OC >> 2], OC & 3);
    }
    const uint32_t re = quick2(pk_even(c), pk_even(u), pk_even(d), pk_even(l), pk_even(r), T2);
    const uint32_t ro = quick2(pk_odd(c), pk_odd(u), pk_odd(d), pk_odd(l), pk_odd(r), T2);
    // pixel k's sign bit at bit 8k + 7: bytes (re.1, ro.1, re.3, ro.3)
    uint32_t m = __builtin_amdgcn_perm(ro, re, 0x07030501u) & (rr < dh ? vmask : 0u);
    const int n = __popc(m);
    const uint64_t b0 = wave_ballot(n & 1), b1 = wave_ballot(n & 2), b2 = wave_ballot(n & 4);
    int pos = nlist + prefix_in_wave(b0) + 2 * prefix_in_wave(b1) + 4 * prefix_in_wave(b2);
    const int px = (rr << 6) + 4 * g;  // list entry r << 6 | c
    while (m) {
      list[pos++] = (uint16_t)(px + (__builtin_ctz(m) >> 3));
      m &= m - 1u;
    }
    nlist += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  }
  return nlist;
}

__device__ __forceinline__ uint32_t pack_key(int x, int y, int s) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
__device__ __forceinline__ int key_x(uint32_t k) { return (int)(k & 0xfffu); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)((k >> 12) & 0xfffu); }
__device__ __forceinline__ int key_s(uint32_t k) { return (int)(k >> 24); }

// k_fast: one wavefront per cell (4 cells per 256-thread workgroup). No workgroup barriers: waves
// are independent and synchronise their own LDS with wave_sync().
// Round 3, measured and rejected: each wavefront running 2-8 consecutive
// cells with the next cell's ROI in flight during the current one -- through a second VGPR set
// (68 -> 109 VGPRs, 7 -> 4 waves per SIMD: 176 -> 198-229 us per 64-image extraction) or by
// LDS-DMA into a second LDS buffer (global_load_lds_dword, 17 dwords per 68-byte row: 206 us at
// one cell per wavefront, 228-275 us at 4-8); LDS sized per launch instead of per pyramid (no
// change). The kernel wants many short wavefronts.
//   1. the cell ROI (<= roi_w_max x roi_h_max) lands in LDS with aligned dword loads;
//   2. OpenCV's antipodal quick test at the lower threshold runs on every detection pixel and the
//      survivors are compacted (ballot + popcount, row-major order kept);
//   3. the full arc strength runs only on the compacted list, full waves;
//   4. strict 3x3 NMS at iniThFAST (then minThFAST for an empty cell) visits only list entries.
__device__ __forceinline__ bool quick_test(const uint8_t* p, int s, int t) {
  // x < v - t  <=>  (x - lo) < 0;  x > v + t  <=>  (hi - x) < 0: the sign bits carry
  // OpenCV's "d &= tab[x] | tab[y]" bits without compares
  const int v = p[0], lo = v - t, hi = v + t;
  int dark = -1, brt = -1;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int x = p[ring_off(k, s)], y = p[ring_off(k + 8, s)];
    dark &= (x - lo) | (y - lo);
    brt &= (hi - x) | (hi - y);
  }
  return (dark | brt) < 0;
}

struct FastLds {
  int rs, roi, m8, list;  // row stride and byte offsets inside one wave's region
  int total;
};
__host__ __device__ inline FastLds fast_lds_layout(int rw_max, int rh_max, int rs_fixed) {
  FastLds f;
  f.rs = rs_fixed ? rs_fixed : (rw_max + 4 + 3) & ~3;
  f.roi = 0;
  f.m8 = (f.rs * rh_max + 15) & ~15;
  f.list = f.m8 + (((rw_max - 4) * (rh_max - 4) + 15) & ~15);
  f.total = f.list + (((rw_max - 6) * (rh_max - 6) * 2 + 15) & ~15);
  return f;
}

// RSC != 0: the ROI row stride is the compile-time constant RSC (68 bytes = 17 banks apart, so
// the rows a wavefront touches spread over the 32 LDS banks) when every ROI fits in 61 columns:
// the 16 ring reads of a pixel are one address plus immediate offsets, the ROI load maps lanes
// with shifts and the row/column split of a detection index is a multiply-shift.
// RSC == 0: any geometry, runtime stride.
template <int RSC>
__global__ __launch_bounds__(512) void k_fast(ExtractArgs a, int cell0, int cell1) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int w = wave_id(), lane = lane_id();
  const int2 blk = xcd_block2d();
  const int cell = cell0 + blk.x * (int)(blockDim.x >> 6) + w;  // cells [cell0, cell1) of this launch
  const int img = blk.y;
  if (cell >= cell1) return;
  const FastLds lay = fast_lds_layout(a.roi_w_max, a.roi_h_max, RSC);
  uint8_t* base = smem + w * lay.total;
  uint8_t* roi = base + lay.roi;
  uint8_t* m8 = base + lay.m8;
  uint16_t* list = reinterpret_cast<uint16_t*>(base + lay.list);
  const int RS = RSC ? RSC : lay.rs;

  const CellDesc cd = a.cells[cell];
  const int pitch = cd.pitch;
  const uint8_t* lev = a.pyr + (long long)img * a.pyr_stride + cd.pyr_off;
  const int rw = cd.rw, rh = cd.rh;
  const int mw = rw - 4, mh = rh - 4, dw = rw - 6, dh = rh - 6;
  int32_t* cnt_out = a.cellcnt + (long long)img * a.ncells + cell;
  if (dw <= 0 || dh <= 0) {
    if (lane == 0) *cnt_out = 0;
    return;
  }
  // 1. ROI -> LDS: dword-aligned columns [x0a, x0a + 4 nw) cover [x0, x0 + rw)
  const int x0a = cd.x0 & ~3, xo = cd.x0 - x0a, nw = (xo + rw + 3) >> 2;
  if constexpr (RSC != 0) {
    // 16-byte loads, 4 lanes per ROI row (<= 61 columns + 3 alignment bytes = 16 dwords); the last
    // quad of a row may read up to 12 bytes past the ROI (row padding / next row / the +256 slack)
    const int nq4 = (nw + 3) >> 2;
    uint4 v[3];  // rh <= 48 rows: 192 quads; unconditional loads (idle lanes re-read quad 0) so
                 // that the three are in flight together
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int i = lane + 64 * k, r = i >> 2, q = i & 3;
      const bool in = r < rh && q < nq4;
      __builtin_memcpy(&v[k], lev + (long long)(cd.y0 + (in ? r : 0)) * pitch + x0a + 16 * (in ? q : 0), 16);
    }
    // the arc-strength map is zeroed while the ROI loads are in flight
    for (int i = lane; i < (mw * mh + 3) >> 2; i += 64) reinterpret_cast<uint32_t*>(m8)[i] = 0u;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int i = lane + 64 * k, r = i >> 2, q = i & 3;
      if (r < rh && q < nq4) {
        uint32_t* d = reinterpret_cast<uint32_t*>(roi + r * RSC + 16 * q);
        d[0] = v[k].x;
        d[1] = v[k].y;
        d[2] = v[k].z;
        d[3] = v[k].w;
      }
    }
    for (int i = lane + 192; i < 4 * rh; i += 64) {  // taller ROIs (rh > 48)
      const int r = i >> 2, q = i & 3;
      if (q < nq4) {
        uint4 v;
        __builtin_memcpy(&v, lev + (long long)(cd.y0 + r) * pitch + x0a + 16 * q, 16);
        uint32_t* d = reinterpret_cast<uint32_t*>(roi + r * RSC + 16 * q);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
    }
  } else {
    for (int i0 = 0; i0 < nw * rh; i0 += 8 * 64) {  // up to 8 dword loads per lane in flight
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = i0 + lane + 64 * k;
        if (i < nw * rh) {
          const int r = i / nw, c = i - r * nw;
          v[k] = *reinterpret_cast<const uint32_t*>(lev + (long long)(cd.y0 + r) * pitch + x0a + 4 * c);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = i0 + lane + 64 * k;
        if (i < nw * rh) {
          const int r = i / nw, c = i - r * nw;
          *reinterpret_cast<uint32_t*>(roi + r * RS + 4 * c) = v[k];
        }
      }
    }
  }
  // list entries: detection pixel (r, c) as r << 6 | c on the constant-stride path (every ROI
  // there is at most 61 columns wide), as r * dw + c on the generic one
  auto dec_rc = [&](int q, int& r, int& c) {
    if constexpr (RSC != 0) {
      r = q >> 6;
      c = q & 63;
    } else {
      r = q / dw;
      c = q - r * dw;
    }
  };
  if constexpr (RSC == 0)
    for (int i = lane; i < (mw * mh + 3) >> 2; i += 64) reinterpret_cast<uint32_t*>(m8)[i] = 0u;
  wave_sync();
  const uint8_t* R = roi + xo;  // pixel (r, c) of the ROI at R[r * RS + c]
  uint32_t* out = a.cand + (long long)img * a.cand_stride + cd.slot;
  int count = 0;
  // ORBextractor.cc:812-819: FAST at iniThFAST; only a cell left empty runs again at minThFAST.
  // Each pass filters, scores and suppresses at its own threshold, so the arc strengths of a
  // textured cell are computed for the iniThFAST corners only. The arc strength M of a pixel does
  // not depend on the threshold, so m8 entries of the first pass stay valid in the second.
  for (int pass = 0; pass < 2; pass++) {
    const int t = min(max(pass == 0 ? a.ini_th : a.min_th, 0), 255);
    if (pass == 1) {
      if (t == min(max(a.ini_th, 0), 255)) break;  // the same threshold finds the same nothing
      wave_sync();  // every lane is done with pass 0's list
    }
    // 2a. OpenCV's first two antipodal pairs (ring 0/8 = dy +-3, ring 4/12 = dx +-3) at t in
    //     packed 16-bit halves (four pixels per lane on the constant-stride path, two otherwise):
    //     dark <=> max(min(u,d), min(l,r)) < v - t, bright <=> min(max(u,d), max(l,r)) > v + t.
    //     Survivors are compacted in row-major order.
    const uint32_t T2 = (uint32_t)t * 0x10001u;
    int nlist = 0;
    if constexpr (RSC != 0) {
      if (dw <= 32) {
        switch (xo) {
          case 0: nlist = fast_prefilter4_g8<RSC, 0>(roi, dw, dh, T2, list); break;
          case 1: nlist = fast_prefilter4_g8<RSC, 1>(roi, dw, dh, T2, list); break;
          case 2: nlist = fast_prefilter4_g8<RSC, 2>(roi, dw, dh, T2, list); break;
          default: nlist = fast_prefilter4_g8<RSC, 3>(roi, dw, dh, T2, list); break;
        }
      } else {
        switch (xo) {
          case 0: nlist = fast_prefilter4<RSC, 0>(roi, dw, dh, T2, list); break;
          case 1: nlist = fast_prefilter4<RSC, 1>(roi, dw, dh, T2, list); break;
          case 2: nlist = fast_prefilter4<RSC, 2>(roi, dw, dh, T2, list); break;
          default: nlist = fast_prefilter4<RSC, 3>(roi, dw, dh, T2, list); break;
        }
      }
    } else {
      const int pw = (dw + 1) >> 1;
      for (int q0 = 0; q0 < pw * dh; q0 += 64) {
        const int q = q0 + lane;
        bool p0 = false, p1 = false;
        int px = 0;
        if (q < pw * dh) {
          const int rr = q / pw;
          const int cc = 2 * (q - rr * pw);
          px = rr * dw + cc;
          const uint8_t* p = R + (rr + 3) * RS + (cc + 3);
          const uint32_t c = pack2(p[0], p[1]);
          const uint32_t u = pack2(p[3 * RS], p[3 * RS + 1]), d = pack2(p[-3 * RS], p[-3 * RS + 1]);
          const uint32_t r = pack2(p[3], p[4]), l = pack2(p[-3], p[-2]);
          const uint32_t X = pk_max_u16(pk_min_u16(u, d), pk_min_u16(l, r));
          const uint32_t Y = pk_min_u16(pk_max_u16(u, d), pk_max_u16(l, r));
          const uint32_t res = pk_sub16(X, pk_sub16(c, T2)) | pk_sub16(pk_add16(c, T2), Y);
          p0 = (res & 0x8000u) != 0;
          p1 = (res & 0x80000000u) != 0 && cc + 1 < dw;
        }
        const uint64_t b0 = wave_ballot(p0), b1 = wave_ballot(p1);
        const int pos = nlist + prefix_in_wave(b0) + prefix_in_wave(b1);
        if (p0) list[pos] = (uint16_t)px;
        if (p1) list[pos + (p0 ? 1 : 0)] = (uint16_t)(px + 1);
        nlist += __popcll(b0) + __popcll(b1);
      }
    }
    wave_sync();
    // 2b+3. on the survivors, two list entries per lane in packed 16-bit halves: the arc strength
    //     (OpenCV cornerScore + 1) of the corners at t goes to m8 and, compacted in order, back
    //     into the list
    int ncorner = 0;
    for (int j0 = 0; j0 < nlist; j0 += 128) {
      const int ja = j0 + 2 * lane, jb = ja + 1;
      int qa = 0, qb = 0;
      uint32_t m = 0;
      if (ja < nlist) {
        qa = list[ja];
        qb = jb < nlist ? list[jb] : qa;
        int ra, ca, rb, cb;
        dec_rc(qa, ra, ca);
        dec_rc(qb, rb, cb);
        const uint8_t* pa = R + (ra + 3) * RS + (ca + 3);
        const uint8_t* pb = R + (rb + 3) * RS + (cb + 3);
        m = arc_strength_pk(pa, pb, RS, t);
        const int ma = (int)(m & 0xffffu), mb = (int)(m >> 16);
        if (ma) m8[(ra + 1) * mw + (ca + 1)] = (uint8_t)min(ma, 255);
        if (mb && jb < nlist) m8[(rb + 1) * mw + (cb + 1)] = (uint8_t)min(mb, 255);
      }
      const bool ka = ja < nlist && (m & 0xffffu) != 0, kb = jb < nlist && (m >> 16) != 0;
      const uint64_t b0 = wave_ballot(ka), b1 = wave_ballot(kb);
      wave_sync();  // every lane has read list[j0 .. j0+127] before it is overwritten
      const int pos = ncorner + prefix_in_wave(b0) + prefix_in_wave(b1);
      if (ka) list[pos] = (uint16_t)qa;
      if (kb) list[pos + (ka ? 1 : 0)] = (uint16_t)qb;
      ncorner += __popcll(b0) + __popcll(b1);
    }
    wave_sync();
    // 4. NMS over the corners at t (out-of-region neighbours and non-corners score 0)
    for (int j0 = 0; j0 < ncorner; j0 += 64) {
      const int j = j0 + lane;
      bool keep = false;
      int rr = 0, cc = 0, sc = 0;
      if (j < ncorner) {
        const int q = list[j];
        dec_rc(q, rr, cc);
        const uint8_t* mp = m8 + (rr + 1) * mw + (cc + 1);
        const int m = mp[0];
        // score m - 1 beats every neighbour's (mn >= t + 1 ? mn - 1 : 0) exactly when m > mn for
        // all 8 neighbours and m >= 2: a neighbour below t + 1 (a corner of an earlier pass at a
        // lower threshold or none) is below m too, and scores 0
        const int mn = max(max(max(max((int)mp[-mw - 1], (int)mp[-mw]), max((int)mp[-mw + 1], (int)mp[-1])),
                               max(max((int)mp[1], (int)mp[mw - 1]), (int)mp[mw])), (int)mp[mw + 1]);
        sc = m - 1;
        keep = m >= max(t + 1, 2) && m > mn;
      }
      const uint64_t bal = wave_ballot(keep);
      if (keep) out[count + prefix_in_wave(bal)] = pack_key(cc + 3 + cd.ox, rr + 3 + cd.oy, sc);
      count += __popcll(bal);
    }
    if (count > 0) break;  // ORBextractor.cc:815-819: minThFAST only for an empty cell
  }
  if (lane == 0) *cnt_out = count;
}

// ---------------------------------------------------------------------------------------------
// k_octree: DistributeOctTree (ORBextractor.cc:542-766) for one (image, level).
//
// The reference keeps a std::list of nodes; every full pass divides every node with >1 key and
// push_front()s its non-empty children n1..n4, so after a pass the list is
//   reverse(children in creation order) ++ (single-key nodes in their old order).
// A refinement round divides the nodes created in the previous pass/round with >1 key in
// descending (size, creation order) -- the reference sorts (size, pointer) pairs; SURVEY C.1 --
// stopping as soon as the list reaches N; its list is
//   reverse(children of the divided nodes, in processing order) ++ (old list minus divided).
// Both are computed with block scans; each node's keys stay one contiguous segment, partitioned
// stably by one wavefront per divided node (ballot + popcount).
// k_octree's LDS scalars: wave sums of the block scans in misc[0 .. NW), scalars from
// misc[OCT_MISC_SCALAR]; OCT_MISC_INTS ints in all (up to 16 wavefronts: 1024 threads)
#define OCT_MISC_SCALAR 16
#define OCT_MISC_INTS 32
struct ONode {
  int16_t x0, y0, x1, y1;
  int32_t begin, count, seq, flags;  // flags: bit0 = key buffer (0: A, 1: B), bit1 = in R set
};


__device__ __forceinline__ int child_of(uint32_t key, int mx, int my) {
  return (key_x(key) >= mx ? 1 : 0) | (key_y(key) >= my ? 2 : 0);
}

// Count the keys of `nd` falling in each of its 4 DivideNode children (wave-level).
__device__ __forceinline__ int4 wave_child_counts(const ONode& nd, const uint32_t* ka, const uint32_t* kb) {
  const uint32_t* src = (nd.flags & 1) ? kb : ka;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  for (int i0 = 0; i0 < nd.count; i0 += 64) {
    const int i = i0 + lane_id();
    const int ch = i < nd.count ? child_of(src[nd.begin + i], mx, my) : -1;
    c0 += __popcll(wave_ballot(ch == 0));
    c1 += __popcll(wave_ballot(ch == 1));
    c2 += __popcll(wave_ballot(ch == 2));
    c3 += __popcll(wave_ballot(ch == 3));
  }
  return make_int4(c0, c1, c2, c3);
}

// Stable 4-way partition of the node's keys into the other buffer (children contiguous, n1..n4).
__device__ __forceinline__ void wave_child_partition(const ONode& nd, int4 cnt, uint32_t* ka, uint32_t* kb) {
  const uint32_t* src = (nd.flags & 1) ? kb : ka;
  uint32_t* dst = (nd.flags & 1) ? ka : kb;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  int o0 = nd.begin, o1 = o0 + cnt.x, o2 = o1 + cnt.y, o3 = o2 + cnt.z;
  for (int i0 = 0; i0 < nd.count; i0 += 64) {
    const int i = i0 + lane_id();
    uint32_t key = 0;
    int ch = -1;
    if (i < nd.count) {
      key = src[nd.begin + i];
      ch = child_of(key, mx, my);
    }
    const uint64_t b0 = wave_ballot(ch == 0), b1 = wave_ballot(ch == 1), b2 = wave_ballot(ch == 2),
                   b3 = wave_ballot(ch == 3);
    if (ch == 0) dst[o0 + prefix_in_wave(b0)] = key;
    if (ch == 1) dst[o1 + prefix_in_wave(b1)] = key;
    if (ch == 2) dst[o2 + prefix_in_wave(b2)] = key;
    if (ch == 3) dst[o3 + prefix_in_wave(b3)] = key;
    o0 += __popcll(b0);
    o1 += __popcll(b1);
    o2 += __popcll(b2);
    o3 += __popcll(b3);
  }
}

// Thread-serial forms for small nodes (count <= ExtractArgs::oct_small, default OCT_SMALL): one lane
// walks the whole segment.
#ifndef OCT_SMALL  // (a build option for the threshold's sweep: profiles/r5_octree_passes.txt)
#define OCT_SMALL 48
#endif
#define OCT_SMALL_MAX 128  // (the host clamps oct_small to it)
// Four keys per step (four independent loads in flight); the four counts / offsets are packed in
// the bytes of one register (count <= oct_small <= OCT_SMALL_MAX < 256), not a dynamically indexed array.
__device__ __forceinline__ int4 serial_child_counts(const ONode& nd, const uint32_t* ka, const uint32_t* kb) {
  const uint32_t* src = ((nd.flags & 1) ? kb : ka) + nd.begin;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  uint32_t c = 0;
  if (nd.count <= 16) {  // every load in flight at once
    uint32_t key[16];
#pragma unroll
    for (int j = 0; j < 16; j++) key[j] = j < nd.count ? src[j] : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++)
      if (j < nd.count) c += 1u << (8 * child_of(key[j], mx, my));
    return make_int4((int)(c & 255u), (int)((c >> 8) & 255u), (int)((c >> 16) & 255u), (int)(c >> 24));
  }
  int i = 0;
  for (; i + 4 <= nd.count; i += 4) {
    const uint32_t k0 = src[i], k1 = src[i + 1], k2 = src[i + 2], k3 = src[i + 3];
    c += (1u << (8 * child_of(k0, mx, my))) + (1u << (8 * child_of(k1, mx, my))) +
         (1u << (8 * child_of(k2, mx, my))) + (1u << (8 * child_of(k3, mx, my)));
  }
  for (; i < nd.count; i++) c += 1u << (8 * child_of(src[i], mx, my));
  return make_int4((int)(c & 255u), (int)((c >> 8) & 255u), (int)((c >> 16) & 255u), (int)(c >> 24));
}

__device__ __forceinline__ void serial_child_partition(const ONode& nd, int4 cnt, uint32_t* ka, uint32_t* kb) {
  const uint32_t* src = ((nd.flags & 1) ? kb : ka) + nd.begin;
  uint32_t* dst = ((nd.flags & 1) ? ka : kb) + nd.begin;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  uint32_t o = ((uint32_t)cnt.x << 8) | ((uint32_t)(cnt.x + cnt.y) << 16) | ((uint32_t)(cnt.x + cnt.y + cnt.z) << 24);
  auto put = [&](uint32_t key) {
    const int sh = 8 * child_of(key, mx, my);
    dst[(o >> sh) & 255u] = key;
    o += 1u << sh;
  };
  if (nd.count <= 16) {  // every load in flight at once
    uint32_t key[16];
#pragma unroll
    for (int j = 0; j < 16; j++) key[j] = j < nd.count ? src[j] : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++)
      if (j < nd.count) put(key[j]);
    return;
  }
  int i = 0;
  for (; i + 4 <= nd.count; i += 4) {
    const uint32_t k0 = src[i], k1 = src[i + 1], k2 = src[i + 2], k3 = src[i + 3];
    put(k0);
    put(k1);
    put(k2);
    put(k3);
  }
  for (; i < nd.count; i++) put(src[i]);
}

// Count + stable partition in one walk for the full passes, the keys read once into registers:
// a wavefront for a large node (up to 64 * OCT_WJ keys), a thread for a small one (up to OCT_SJ).
#define OCT_WJ 16
#define OCT_SJ 16
__device__ __forceinline__ int4 wave_child_split(const ONode& nd, uint32_t* ka, uint32_t* kb) {
  if (nd.count > 64 * OCT_WJ) {
    const int4 c4 = wave_child_counts(nd, ka, kb);
    wave_child_partition(nd, c4, ka, kb);
    return c4;
  }
  const uint32_t* src = ((nd.flags & 1) ? kb : ka) + nd.begin;
  uint32_t* dst = ((nd.flags & 1) ? ka : kb) + nd.begin;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  const int lane = lane_id();
  uint32_t key[OCT_WJ];
  int ch[OCT_WJ];
#pragma unroll
  for (int j = 0; j < OCT_WJ; j++) {
    const int i = 64 * j + lane;
    key[j] = i < nd.count ? src[i] : 0u;
  }
  int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
  for (int j = 0; j < OCT_WJ; j++) {
    if (64 * j >= nd.count) break;
    ch[j] = 64 * j + lane < nd.count ? child_of(key[j], mx, my) : -1;
    c0 += __popcll(wave_ballot(ch[j] == 0));
    c1 += __popcll(wave_ballot(ch[j] == 1));
    c2 += __popcll(wave_ballot(ch[j] == 2));
    c3 += __popcll(wave_ballot(ch[j] == 3));
  }
  int o0 = 0, o1 = c0, o2 = c0 + c1, o3 = c0 + c1 + c2;
#pragma unroll
  for (int j = 0; j < OCT_WJ; j++) {
    if (64 * j >= nd.count) break;
    const uint64_t b0 = wave_ballot(ch[j] == 0), b1 = wave_ballot(ch[j] == 1), b2 = wave_ballot(ch[j] == 2),
                   b3 = wave_ballot(ch[j] == 3);
    if (ch[j] == 0) dst[o0 + prefix_in_wave(b0)] = key[j];
    if (ch[j] == 1) dst[o1 + prefix_in_wave(b1)] = key[j];
    if (ch[j] == 2) dst[o2 + prefix_in_wave(b2)] = key[j];
    if (ch[j] == 3) dst[o3 + prefix_in_wave(b3)] = key[j];
    o0 += __popcll(b0);
    o1 += __popcll(b1);
    o2 += __popcll(b2);
    o3 += __popcll(b3);
  }
  return make_int4(c0, c1, c2, c3);
}

__device__ __forceinline__ int4 serial_child_split(const ONode& nd, uint32_t* ka, uint32_t* kb) {
  if (nd.count > OCT_SJ) {
    const int4 c4 = serial_child_counts(nd, ka, kb);
    serial_child_partition(nd, c4, ka, kb);
    return c4;
  }
  const uint32_t* src = ((nd.flags & 1) ? kb : ka) + nd.begin;
  uint32_t* dst = ((nd.flags & 1) ? ka : kb) + nd.begin;
  const int mx = nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1), my = nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1);
  uint32_t key[OCT_SJ];
#pragma unroll
  for (int j = 0; j < OCT_SJ; j++) key[j] = j < nd.count ? src[j] : 0u;
  uint32_t c = 0;  // four 8-bit counts
#pragma unroll
  for (int j = 0; j < OCT_SJ; j++)
    if (j < nd.count) c += 1u << (8 * child_of(key[j], mx, my));
  const uint32_t c0 = c & 255u, c1 = (c >> 8) & 255u, c2 = (c >> 16) & 255u;
  uint32_t o = (c0 << 8) | ((c0 + c1) << 16) | ((c0 + c1 + c2) << 24);
#pragma unroll
  for (int j = 0; j < OCT_SJ; j++)
    if (j < nd.count) {
      const int sh = 8 * child_of(key[j], mx, my);
      dst[(o >> sh) & 255u] = key[j];
      o += 1u << sh;
    }
  return make_int4((int)c0, (int)c1, (int)c2, (int)(c >> 24));
}

__device__ __forceinline__ ONode make_child(const ONode& p, int c, int begin, int count, int seq) {
  const int mx = p.x0 + ((p.x1 - p.x0 + 1) >> 1), my = p.y0 + ((p.y1 - p.y0 + 1) >> 1);
  ONode n;
  n.x0 = (int16_t)((c & 1) ? mx : p.x0);
  n.x1 = (int16_t)((c & 1) ? p.x1 : mx);
  n.y0 = (int16_t)((c & 2) ? my : p.y0);
  n.y1 = (int16_t)((c & 2) ? p.y1 : my);
  n.begin = begin;
  n.count = count;
  n.seq = seq;
  n.flags = ((p.flags & 1) ^ 1) | (count > 1 ? 2 : 0);
  return n;
}

__device__ __forceinline__ int nonempty4(int4 c) {
  return (c.x > 0) + (c.y > 0) + (c.z > 0) + (c.w > 0);
}
__device__ __forceinline__ int multi4(int4 c) {
  return (c.x > 1) + (c.y > 1) + (c.z > 1) + (c.w > 1);
}
__device__ __forceinline__ int comp4(int4 c, int k) {
  return k == 0 ? c.x : k == 1 ? c.y : k == 2 ? c.z : c.w;
}

// The nodes of list positions [0, m) (position p -> node index idx(p)) holding more than `small`
// keys, dealt round-robin over the block's NW wavefronts in position order: each wavefront reads the
// counts of 64 positions at a time (one LDS read per lane) and walks the ballot of the big ones, so
// no wavefront steps through the small nodes one dependent read at a time.
template <int NW, typename Idx, typename F>
__device__ __forceinline__ void for_big_nodes(const ONode* L, int m, int small, Idx idx, F f) {
  const int w = wave_id(), lane = lane_id();
  int ord = 0;
  for (int c0 = 0; c0 < m; c0 += 64) {
    const int p = c0 + lane;
    const bool big = p < m && L[idx(p)].count > small;
    uint64_t bal = wave_ballot(big);
    while (bal) {
      const int b = __builtin_ctzll(bal);
      bal &= bal - 1;
      if (ord % NW == w) f(c0 + b);
      ord++;
    }
  }
}

// Phase clocks of k_octree (profiling builds only, -DORBFE_OCT_PROF=1, read by
// profiles/scripts/r5_octree_prof.py through orbfe_debug_octree_prof): per (image < 64, level < 16)
// wall_clock64 at the kernel start, after the cell-count scan, the gather, the initial nodes, the
// first refinement round, the loop end and the end, then n | passes << 24 | rounds << 32 | S << 48;
// slots 8-13 inside the first refinement round (after the flag scan, the sort, the child counts,
// the stop scan, the partition, the round), 14-15 inside the first full pass (after the splits,
// after the scan).
#ifdef ORBFE_OCT_PROF
__device__ unsigned long long g_oct_prof[64 * 16 * 16];
#define OCT_MARK(k, v) \
  do { if (threadIdx.x == 0 && blockIdx.y < 64 && l < 16) g_oct_prof[(blockIdx.y * 16 + l) * 16 + (k)] = (v); } while (0)
#else
#define OCT_MARK(k, v) do { } while (0)
#endif
#ifdef ORBFE_OCT_PROF_PASS  // slots 8-11 then time the sub-steps of that full pass instead
#define OCT_RMARK(k, v) do { } while (0)
#define OCT_PMARK(k, v) do { if (n_passes == ORBFE_OCT_PROF_PASS) OCT_MARK(k, v); } while (0)
#else
#define OCT_RMARK(k, v) OCT_MARK(k, v)
#define OCT_PMARK(k, v) do { } while (0)
#endif

template <bool LDSK, int NT>
__device__ __forceinline__ void octree_run(const ExtractArgs& a, uint8_t* smem, int l, int n, uint32_t* ka,
                                           uint32_t* kb) {
  constexpr int NW = NT / 64;
  const int img = blockIdx.y;
  const int t = threadIdx.x, w = wave_id(), lane = lane_id();
  const int NC = a.node_cap, SC = a.sort_cap, SA = a.scan_cap;
  const int SMALL = a.oct_small;
  ONode* nodes0 = reinterpret_cast<ONode*>(smem);
  ONode* nodes1 = nodes0 + NC;
  int4* cc = reinterpret_cast<int4*>(nodes1 + NC);
  int* sa = reinterpret_cast<int*>(cc + NC);
  int* sb = sa + SA;
  int* sx = sb + SA;
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(sx + SA);
  int* misc = reinterpret_cast<int*>(sk + SC);  // [0..NW) scan wave sums, [OCT_MISC_SCALAR..] scalars
  const LevelDesc ld = a.levels[l];
  const int N = ld.budget;
  const uint32_t* cand = a.cand + (long long)img * a.cand_stride;
  uint32_t* out = a.lvlkeys + (long long)img * a.lvlkey_stride + ld.key_begin;
  int32_t* out_n = a.lvlcnt + (long long)img * a.nlevels + l;

  // 1. gather this level's FAST candidates in cell order (ComputeKeyPointsOctTree :821-829):
  //    sa = exclusive prefix of the cell counts, sx = cell slots (filled by the caller); a thread
  //    per cell copies the cell's keys, four loads in flight
  const int ncells = ld.ncells;
  for (int c = t; c < ncells; c += NT) {
    const int b0 = sa[c], cnt = (c + 1 < ncells ? sa[c + 1] : n) - b0;
    const uint32_t* src = cand + sx[c];
    int k = 0;
    for (; k + 4 <= cnt; k += 4) {
      const uint32_t v0 = src[k], v1 = src[k + 1], v2 = src[k + 2], v3 = src[k + 3];
      ka[b0 + k] = v0;
      ka[b0 + k + 1] = v1;
      ka[b0 + k + 2] = v2;
      ka[b0 + k + 3] = v3;
    }
    for (; k < cnt; k++) ka[b0 + k] = src[k];
  }
  __syncthreads();
  OCT_MARK(2, wall_clock64());

  // 2. initial nodes (:555-588): key -> vpIniNodes[(size_t)(x / hX)], stable, all 4 waves:
  //    wave w counts then places the keys of its quarter; bucket offsets in between
  const int nini = ld.nini;
  const float hx = ld.hx;
  auto ini_node = [&](uint32_t key) -> int {  // (size_t)(kp.pt.x / hX) (:575)
    const int x = key_x(key);
    if (nini > 8) return (int)((float)x / hx);
    int b = 0;
#pragma unroll
    for (int k = 1; k < 8; k++) b += (k < nini && x >= ld.ini_thr[k]) ? 1 : 0;
    return b;
  };
  int* bcnt = reinterpret_cast<int*>(sk);  // [NW][nini] counts, then [NW][nini] offsets
  int* boff = bcnt + NW * nini;
  const int R = ((n + NW - 1) / NW + 63) & ~63;
  const int wbeg = min(w * R, n), wend = min(wbeg + R, n);
  // the wave's keys and their initial nodes stay in registers for both walks (one LDS read and one
  // bucket per key) when the quarter has at most 64 * INI_J keys
  constexpr int INI_J = NT >= 1024 ? 8 : 24;  // (16 wavefronts: 8 rows cache 8,192 keys)
  const bool cached = wend - wbeg <= 64 * INI_J;
  uint32_t kr[INI_J];
  int br[INI_J];
  const int nj = (wend - wbeg + 63) >> 6;  // register rows this wave uses (wave-uniform)
  if (cached) {
    // only the rows the wave's keys fill, the bucket by compares against the host thresholds
    // (the division form only for nIni > 8), so the unrolled loop carries no dead rows
#pragma unroll
    for (int j = 0; j < INI_J; j++) br[j] = -1;
    if (nini <= 8) {
#pragma unroll
      for (int j = 0; j < INI_J; j++) {
        if (j >= nj) break;
        const int i = wbeg + 64 * j + lane;
        kr[j] = i < wend ? ka[i] : 0u;
        const int x = key_x(kr[j]);
        int b = 0;
#pragma unroll
        for (int k = 1; k < 8; k++) b += (k < nini && x >= ld.ini_thr[k]) ? 1 : 0;
        br[j] = i < wend ? b : -1;
      }
    } else {
#pragma unroll
      for (int j = 0; j < INI_J; j++) {
        if (j >= nj) break;
        const int i = wbeg + 64 * j + lane;
        kr[j] = i < wend ? ka[i] : 0u;
        br[j] = i < wend ? (int)((float)key_x(kr[j]) / hx) : -1;
      }
    }
  }
  for (int bkt = 0; bkt < nini; bkt++) {
    int cnt = 0;
    if (cached) {
#pragma unroll
      for (int j = 0; j < INI_J; j++) {
        if (j >= nj) break;
        cnt += __popcll(wave_ballot(br[j] == bkt));
      }
    } else {
      for (int i0 = wbeg; i0 < wend; i0 += 64) {
        const int i = i0 + lane;
        const bool in = i < wend && ini_node(ka[i]) == bkt;
        cnt += __popcll(wave_ballot(in));
      }
    }
    if (lane == 0) bcnt[w * nini + bkt] = cnt;
  }
  __syncthreads();
  if (nini * NW <= 64) {  // bucket-major offsets by one wavefront's scan (lane q: bucket q / NW, wave q % NW)
    if (w == 0) {
      const int q = lane, bkt = q / NW, ww = q - bkt * NW;
      const bool in = q < nini * NW;
      const int v = in ? bcnt[ww * nini + bkt] : 0;
      int inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const int first = __shfl(inc - v, min(bkt, 63 / NW) * NW, 64);  // the bucket's first exclusive sum
      if (in) {
        boff[ww * nini + bkt] = inc - v;
        if (ww == NW - 1) sb[bkt] = inc - first;
      }
    }
  } else if (t == 0) {
    int run = 0;
    for (int bkt = 0; bkt < nini; bkt++) {
      sb[bkt] = 0;
      for (int ww = 0; ww < NW; ww++) {
        boff[ww * nini + bkt] = run;
        run += bcnt[ww * nini + bkt];
        sb[bkt] += bcnt[ww * nini + bkt];
      }
    }
  }
  __syncthreads();
  for (int bkt = 0; bkt < nini; bkt++) {
    int run = boff[w * nini + bkt];
    if (cached) {
#pragma unroll
      for (int j = 0; j < INI_J; j++) {
        if (j >= nj) break;
        const bool in = br[j] == bkt;
        const uint64_t bal = wave_ballot(in);
        if (in) kb[run + prefix_in_wave(bal)] = kr[j];
        run += __popcll(bal);
      }
    } else {
      for (int i0 = wbeg; i0 < wend; i0 += 64) {
        const int i = i0 + lane;
        uint32_t key = 0;
        bool in = false;
        if (i < wend) {
          key = ka[i];
          in = ini_node(key) == bkt;
        }
        const uint64_t bal = wave_ballot(in);
        if (in) kb[run + prefix_in_wave(bal)] = key;
        run += __popcll(bal);
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    int S = 0, run = 0;
    for (int b = 0; b < nini; b++) {
      const int cnt = sb[b];
      if (cnt > 0) {
        ONode nd;
        nd.x0 = (int16_t)(int)(hx * (float)b);
        nd.x1 = (int16_t)(int)(hx * (float)(b + 1));
        nd.y0 = 0;
        nd.y1 = (int16_t)ld.rel_h;
        nd.begin = run;
        nd.count = cnt;
        nd.seq = b;
        nd.flags = 1;  // keys in buffer B
        nodes0[S++] = nd;
      }
      run += cnt;
    }
    misc[OCT_MISC_SCALAR] = S;
  }
  __syncthreads();

  int S = misc[OCT_MISC_SCALAR];
  int cur = 0;
  bool refine = false;
  OCT_MARK(3, wall_clock64());
  int n_passes = 0, n_rounds = 0;
  for (int iter = 0; iter < 4 * NC + 64; iter++) {
    ONode* Lc = cur ? nodes1 : nodes0;
    ONode* Ln = cur ? nodes0 : nodes1;
    const int prevS = S;
    if (!refine) {
      n_passes++;
#ifdef ORBFE_OCT_PROF_PASS  // (profiling builds: marks 14/15 bracket full pass ORBFE_OCT_PROF_PASS)
      if (n_passes == ORBFE_OCT_PROF_PASS) OCT_MARK(14, wall_clock64());
#endif
      // ---- full pass (:603-668) ----
      // each node's split and its scan inputs by whoever splits it (a thread for <= oct_small
      // keys, a wavefront above): children (sa), kept single-key nodes (sb), multi-key children (sx)
      for (int i = t; i < S; i += NT) {
        const ONode nd = Lc[i];
        if (nd.count > SMALL) continue;
        const bool par = nd.count > 1;
        const int4 c4 = par ? serial_child_split(nd, ka, kb) : make_int4(0, 0, 0, 0);
        if (par) cc[i] = c4;
        sa[i] = par ? nonempty4(c4) : 0;
        sb[i] = par ? 0 : 1;
        sx[i] = par ? multi4(c4) : 0;
      }
      OCT_PMARK(8, wall_clock64());
#ifdef ORBFE_OCT_PROF_PASS
      unsigned long long split_cyc = 0, split_n = 0;
#endif
      for_big_nodes<NW>(Lc, S, SMALL, [](int p) { return p; }, [&](int i) {
#ifdef ORBFE_OCT_PROF_PASS
        const unsigned long long c0 = clock64();
        const int4 c4 = wave_child_split(Lc[i], ka, kb);
        split_cyc += clock64() - c0;
        split_n += (unsigned long long)Lc[i].count << 16 | 1ull;
#else
        const int4 c4 = wave_child_split(Lc[i], ka, kb);
#endif
        if (lane == 0) {
          cc[i] = c4;
          sa[i] = nonempty4(c4);
          sb[i] = 0;
          sx[i] = multi4(c4);
        }
      });
      OCT_PMARK(9, wall_clock64());
#ifdef ORBFE_OCT_PROF_PASS  // wave 0's shader clocks inside its wave splits, its keys << 16 | splits
      OCT_PMARK(12, split_cyc);
      OCT_PMARK(13, split_n);
#endif
      __syncthreads();
      OCT_PMARK(10, wall_clock64());
#ifndef ORBFE_OCT_PROF_PASS
      if (n_passes == 1) OCT_MARK(14, wall_clock64());
#endif
      // (sk is free during full passes: its first 12 ints hold the scan's wave sums)
      const int3 tot3 = block_scan_excl3_n<NT>(sa, sb, sx, S, reinterpret_cast<int*>(sk));
#ifndef ORBFE_OCT_PROF_PASS
      if (n_passes == 1) OCT_MARK(15, wall_clock64());
#endif
      OCT_PMARK(11, wall_clock64());
      const int T = tot3.x, NP = tot3.y, nexp = tot3.z;
      for (int i = t; i < S; i += NT) {
        const ONode nd = Lc[i];
        if (nd.count > 1) {
          const int4 c4 = cc[i];
          int e = sa[i], off = nd.begin;
          for (int k = 0; k < 4; k++) {
            const int ck = comp4(c4, k);
            if (ck > 0) {
              Ln[T - 1 - e] = make_child(nd, k, off, ck, e);
              e++;
            }
            off += ck;
          }
        } else {
          ONode m = nd;
          m.flags &= 1;
          Ln[T + sb[i]] = m;
        }
      }
      S = T + NP;
      cur ^= 1;
      __syncthreads();
#ifdef ORBFE_OCT_PROF_PASS
      if (n_passes == ORBFE_OCT_PROF_PASS) OCT_MARK(15, wall_clock64());
#endif
      if (S >= N || S == prevS) break;
      if (S + nexp * 3 > N) refine = true;
    } else {
      if (n_rounds++ == 0) OCT_MARK(4, wall_clock64());
      // ---- refinement round (:679-740) ----
      for (int i = t; i < S; i += NT) sa[i] = (Lc[i].flags & 2) ? 1 : 0;
      __syncthreads();
      const int nR = block_scan_excl_n<NT>(sa, S, misc);
      if (n_rounds == 1) OCT_RMARK(8, wall_clock64());
      int P2 = 1;
      while (P2 < nR) P2 <<= 1;
      if (nR > 1024) {
        for (int i = t; i < P2; i += NT) sk[i] = 0ull;
        __syncthreads();
      }
      for (int i = t; i < S; i += NT) {
        const ONode nd = Lc[i];
        if (nd.flags & 2)
          sk[sa[i]] = ((unsigned long long)nd.count << 40) | ((unsigned long long)nd.seq << 20) |
                      (unsigned long long)i;
      }
      __syncthreads();
      if (nR <= 1024) {
        // rank sort, descending (largest (size, creation) first; the keys are distinct): every
        // key counts the larger ones with broadcast LDS reads -- two barriers instead of a
        // bitonic network's log^2
        constexpr int RP = (1024 + NT - 1) / NT;  // keys per thread
        unsigned long long kk[RP];
        int rk[RP];
#pragma unroll
        for (int r = 0; r < RP; r++) {
          const int k = t + NT * r;
          kk[r] = k < nR ? sk[k] : 0ull;
          rk[r] = 0;
        }
        const int per = (nR + NT - 1) / NT;
        int j = 0;
        for (; j + 16 <= nR; j += 16) {  // sixteen broadcast reads in flight
          unsigned long long y[16];
#pragma unroll
          for (int q = 0; q < 16; q++) y[q] = sk[j + q];
#pragma unroll
          for (int r = 0; r < RP; r++)
            if (r == 0 || per > r) {
#pragma unroll
              for (int q = 0; q < 16; q++) rk[r] += y[q] > kk[r];
            }
        }
        for (; j < nR; j++) {
          const unsigned long long y = sk[j];
#pragma unroll
          for (int r = 0; r < RP; r++)
            if (r == 0 || per > r) rk[r] += y > kk[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RP; r++)
          if (t + NT * r < nR) sk[rk[r]] = kk[r];
        __syncthreads();
      } else {
        // bitonic sort, descending: largest (size, creation) first
        for (int k = 2; k <= P2; k <<= 1) {
          for (int j = k >> 1; j > 0; j >>= 1) {
            for (int pidx = t; pidx < (P2 >> 1); pidx += NT) {
              const int i = ((pidx & ~(j - 1)) << 1) | (pidx & (j - 1)), ixj = i + j;  // j is a power of 2
              const unsigned long long x = sk[i], y = sk[ixj];
              if ((i & k) == 0 ? (x < y) : (x > y)) {
                sk[i] = y;
                sk[ixj] = x;
              }
            }
            __syncthreads();
          }
        }
      }
      if (n_rounds == 1) OCT_RMARK(9, wall_clock64());
      // child counts of every candidate, in processing order
      for (int k = t; k < nR; k += NT) {
        const ONode nd = Lc[(int)(sk[k] & 0xfffffull)];
        if (nd.count <= SMALL) cc[k] = serial_child_counts(nd, ka, kb);
      }
      for_big_nodes<NW>(Lc, nR, SMALL, [&](int k) { return (int)(sk[k] & 0xfffffull); }, [&](int k) {
        const int4 c4 = wave_child_counts(Lc[(int)(sk[k] & 0xfffffull)], ka, kb);
        if (lane == 0) cc[k] = c4;
      });
      __syncthreads();
      if (n_rounds == 1) OCT_RMARK(10, wall_clock64());
      for (int k = t; k < nR; k += NT) sa[k] = nonempty4(cc[k]) - 1;
      if (t == 0) misc[OCT_MISC_SCALAR + 1] = nR;
      __syncthreads();
      block_scan_excl_n<NT>(sa, nR, misc);
      for (int k = t; k < nR; k += NT) {
        const int incl = sa[k] + nonempty4(cc[k]) - 1;
        if (prevS + incl >= N) atomicMin(&misc[OCT_MISC_SCALAR + 1], k + 1);  // break at the first k reaching N
      }
      __syncthreads();
      const int nproc = misc[OCT_MISC_SCALAR + 1];
      if (n_rounds == 1) OCT_RMARK(11, wall_clock64());
      for (int i = t; i < S; i += NT) sb[i] = -1;
      __syncthreads();
      for (int k = t; k < nproc; k += NT) sb[(int)(sk[k] & 0xfffffull)] = k;
      __syncthreads();
      // partition the divided nodes' keys
      for (int k = t; k < nproc; k += NT) {
        const ONode nd = Lc[(int)(sk[k] & 0xfffffull)];
        if (nd.count <= SMALL) serial_child_partition(nd, cc[k], ka, kb);
      }
      for_big_nodes<NW>(Lc, nproc, SMALL, [&](int k) { return (int)(sk[k] & 0xfffffull); }, [&](int k) {
        wave_child_partition(Lc[(int)(sk[k] & 0xfffffull)], cc[k], ka, kb);
      });
      for (int k = t; k < nR; k += NT) sx[k] = k < nproc ? nonempty4(cc[k]) : 0;
      __syncthreads();
      if (n_rounds == 1) OCT_RMARK(12, wall_clock64());
      const int T = block_scan_excl_n<NT>(sx, nR, misc);
      for (int i = t; i < S; i += NT) sa[i] = sb[i] < 0 ? 1 : 0;
      __syncthreads();
      const int NK = block_scan_excl_n<NT>(sa, S, misc);
      for (int i = t; i < S; i += NT) {
        const ONode nd = Lc[i];
        const int k = sb[i];
        if (k >= 0) {
          const int4 c4 = cc[k];
          int e = sx[k], off = nd.begin;
          for (int c = 0; c < 4; c++) {
            const int ck = comp4(c4, c);
            if (ck > 0) {
              Ln[T - 1 - e] = make_child(nd, c, off, ck, e);
              e++;
            }
            off += ck;
          }
        } else {
          ONode m = nd;
          m.flags &= 1;
          Ln[T + sa[i]] = m;
        }
      }
      S = T + NK;
      cur ^= 1;
      __syncthreads();
      if (n_rounds == 1) OCT_RMARK(13, wall_clock64());
      if (S >= N || S == prevS) break;
    }
  }

  OCT_MARK(5, wall_clock64());
  if (n_rounds == 0) OCT_MARK(4, wall_clock64());
  // 3. retain the best key of every node, in list order (:744-763; strict '>' keeps the first)
  ONode* Lf = cur ? nodes1 : nodes0;
  for (int i = t; i < S; i += NT) {
    const ONode nd = Lf[i];
    const uint32_t* src = (nd.flags & 1) ? kb : ka;
    uint32_t best = src[nd.begin];
    for (int k = 1; k < nd.count; k++) {
      const uint32_t key = src[nd.begin + k];
      if (key_s(key) > key_s(best)) best = key;
    }
    // back to level coordinates: pt += (minBorderX, minBorderY) (:846-847)
    out[i] = pack_key(key_x(best) + 16, key_y(best) + 16, key_s(best));
  }
  if (t == 0) *out_n = S;
#ifdef ORBFE_OCT_PROF
  __syncthreads();
  OCT_MARK(6, wall_clock64());
  OCT_MARK(7, (unsigned long long)n | ((unsigned long long)n_passes << 24) | ((unsigned long long)n_rounds << 32) |
                  ((unsigned long long)S << 48));
#endif
}


template <int NT>
__global__ __launch_bounds__(NT) void k_octree(ExtractArgs a, int l0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int l = l0 + blockIdx.x, img = blockIdx.y, t = threadIdx.x;  // levels l0 .. l0 + gridDim.x - 1
  const int NC = a.node_cap, SC = a.sort_cap, SA = a.scan_cap;
  int* sa = reinterpret_cast<int*>(smem + (sizeof(ONode) * 2 + sizeof(int4)) * NC);
  int* sx = sa + 2 * SA;
  int* misc = reinterpret_cast<int*>(reinterpret_cast<unsigned long long*>(sx + SA) + SC);
  uint32_t* lds_keys = reinterpret_cast<uint32_t*>(misc + OCT_MISC_INTS);
  OCT_MARK(0, wall_clock64());
  const LevelDesc ld = a.levels[l];
  const int32_t* ccount = a.cellcnt + (long long)img * a.ncells + ld.cell_begin;
  for (int c = t; c < ld.ncells; c += NT) {
    sa[c] = ccount[c];
    sx[c] = a.cells[ld.cell_begin + c].slot;
  }
  __syncthreads();
  const int n = block_scan_excl_n<NT>(sa, ld.ncells, misc);
  OCT_MARK(1, wall_clock64());
  if (n == 0) {
    if (t == 0) a.lvlcnt[(long long)img * a.nlevels + l] = 0;
    return;
  }
  if (n <= a.key_lds_cap) {  // keys in LDS (two ping-pong halves)
    octree_run<true, NT>(a, smem, l, n, lds_keys, lds_keys + a.key_lds_cap);
  } else {  // very large levels: keys in the global scratch buffers
    octree_run<false, NT>(a, smem, l, n, a.keys_a + (long long)img * a.keyscr_stride + ld.cand_begin,
                      a.keys_b + (long long)img * a.keyscr_stride + ld.cand_begin);
  }
}

// ---------------------------------------------------------------------------------------------
#define BS_W 248  // output columns per wavefront strip: lanes 1..62, 4 each (lanes 0 and 63 halo)
#define BS_H 16   // output rows per strip
__device__ __forceinline__ int reflect101(int i, int n) {
  return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

// whole-wavefront lane shifts (DPP wave_shr:1 / wave_shl:1, gfx9): lane i <- lane i-1 / i+1
// (bound_ctrl: the lane without a source, 0 or 63, reads 0 -- a halo lane whose output is
// unused -- and no old value has to be kept in the destination register)
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2v, a) * __builtin_bit_cast(u16x2v, b) +
                                          __builtin_bit_cast(u16x2v, c));
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2v, a) + __builtin_bit_cast(u16x2v, b));
}
// 7-tap [18 34 49 54 49 34 18] over 7 packed rows (each half one column; sums <= 65280 fit u16)
__device__ __forceinline__ uint32_t vtap7(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t r4,
                                          uint32_t r5, uint32_t r6) {
  uint32_t v = pk_mad_u16(r3, 0x00360036u, 0u);
  v = pk_mad_u16(pk_add_u16(r2, r4), 0x00310031u, v);
  v = pk_mad_u16(pk_add_u16(r1, r5), 0x00220022u, v);
  return pk_mad_u16(pk_add_u16(r0, r6), 0x00120012u, v);
}

// k_blur: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of every level (ORBextractor.cc:1083-1084),
// OpenCV's bit-exact fixed-point form out = (sum_j k_j sum_i k_i p_ij + 2^15) >> 16 with
// k = [18, 34, 49, 54, 49, 34, 18]; the sums are exact integers, so the vertical pass may run
// first. One wavefront per 248 x 32 strip, each lane one dword (4 columns) per input row: the
// 7-row window is kept as packed 16-bit (even, odd) column pairs, the vertical taps are v_pk_mad_u16
// (V <= 65280), the neighbours' V come by DPP lane shifts (lanes 0 and 63 are halo), and the
// horizontal taps are 4 v_dot2_u32_u16 per pixel on consecutive column pairs built with v_perm.
// Strips of all levels of all images in one launch.
__global__ __launch_bounds__(256) void k_blur(ExtractArgs a) {
  const int2 blk = xcd_block2d();
  const int img = blk.y, lane = lane_id();
  int strip = blk.x * (int)(blockDim.x >> 6) + wave_id(), l = 0;
  if (strip >= a.blur_strips) return;
  while (l + 1 < a.nlevels && strip >= a.levels[l + 1].tile_begin) l++;
  const LevelDesc ld = a.levels[l];
  strip -= ld.tile_begin;
  // full strips: BS_W columns x BS_H rows. The level's last, narrower column strip (width
  // w - tiles_x * BS_W) splits the wavefront into blur_h groups of 64 / blur_h lanes, each with
  // its own halo lanes and its own band of BS_H rows (the wave shifts below cross a group edge
  // only into halo lanes), so that few lanes idle beside a narrow remainder.
  const int nfull = ld.tiles_x * ((ld.h + BS_H - 1) / BS_H);
  int x, y0, gl, lg;
  if (strip < nfull) {
    const int sx = strip % ld.tiles_x, sy = strip / ld.tiles_x;
    x = sx * BS_W - 4 + 4 * lane;  // this lane's 4 columns
    y0 = sy * BS_H;
    gl = lane;
    lg = 64;
  } else {
    const int H = ld.blur_h;
    lg = 64 / H;
    gl = lane & (lg - 1);
    x = ld.tiles_x * BS_W - 4 + 4 * gl;
    y0 = ((strip - nfull) * H + lane / lg) * BS_H;
  }
  const uint8_t* src = a.pyr + (long long)img * a.pyr_stride + ld.pyr_off;
  uint8_t* dst = a.blur + (long long)img * a.pyr_stride + ld.pyr_off;
  const int w = ld.w, pitch = ld.pitch;
  // columns -4 .. w+7 exist in every row (padding; -3..-1 and w..w+2 hold the reflections)
  const bool cin = x < w + 8;
  const bool out = gl >= 1 && gl <= lg - 2 && x < w;
  // stores through a buffer resource on the level's column -4: 32-bit offsets
  const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(dst - 4, 0, 0x7fffffff, 0x00020000);
  const int wo = y0 * ld.pitch + x + 4;  // this lane's first output row, column x
  auto load_row = [&](int r) {
    return cin ? *reinterpret_cast<const uint32_t*>(src + (long long)reflect101(r, ld.h) * pitch + x) : 0u;
  };
  auto ev = [](uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c020c00u); };  // columns 0, 2
  auto od = [](uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c030c01u); };  // columns 1, 3
  const int yend = min(y0 + BS_H, ld.h);
  const int nrows = y0 < ld.h ? yend - y0 + 6 : 0;  // input rows y0-3 .. yend+2 (<= BS_H + 6)
  // every input row of the strip is loaded up front (fully unrolled: all loads in flight at once,
  // the window below is renamed, not moved)
  uint32_t rowv[BS_H + 6];
#pragma unroll
  for (int i = 0; i < BS_H + 6; i++) rowv[i] = i < nrows ? load_row(y0 - 3 + i) : 0u;
  // the rounding constant 2^15 in one VGPR for the whole strip (not an inline constant; left to
  // the compiler it is rematerialised per row)
  uint32_t seed;
  asm volatile("v_mov_b32 %0, 0x8000" : "=v"(seed));
  uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0, e4 = 0, e5 = 0, e6 = 0;  // window, even columns
  uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0;  // window, odd columns
#pragma unroll
  for (int i = 0; i < BS_H + 6; i++) {
    const uint32_t C = rowv[i];
    e0 = e1; e1 = e2; e2 = e3; e3 = e4; e4 = e5; e5 = e6; e6 = ev(C);
    o0 = o1; o1 = o2; o2 = o3; o3 = o4; o4 = o5; o5 = o6; o6 = od(C);
    if (i < 6 || i >= nrows) continue;
    // vertical: V of columns x, x+2 (VE) and x+1, x+3 (VO)
    const uint32_t VE = vtap7(e0, e1, e2, e3, e4, e5, e6), VO = vtap7(o0, o1, o2, o3, o4, o5, o6);
    const uint32_t LE = from_left(VE), LO = from_left(VO), RE = from_right(VE), RO = from_right(VO);
    // consecutive column pairs P(k) = (V(x+k), V(x+k+1)), k = -3..6
    const uint32_t Pm3 = __builtin_amdgcn_perm(LE, LO, 0x07060100u);  // (V-3, V-2)
    const uint32_t Pm2 = __builtin_amdgcn_perm(LO, LE, 0x07060302u);  // (V-2, V-1)
    const uint32_t Pm1 = __builtin_amdgcn_perm(VE, LO, 0x05040302u);  // (V-1, V0)
    const uint32_t P0 = __builtin_amdgcn_perm(VO, VE, 0x05040100u);   // (V0, V1)
    const uint32_t P1 = __builtin_amdgcn_perm(VE, VO, 0x07060100u);   // (V1, V2)
    const uint32_t P2 = __builtin_amdgcn_perm(VO, VE, 0x07060302u);   // (V2, V3)
    const uint32_t P3 = __builtin_amdgcn_perm(RE, VO, 0x05040302u);   // (V3, V4)
    const uint32_t P4 = __builtin_amdgcn_perm(RO, RE, 0x05040100u);   // (V4, V5)
    const uint32_t P5 = __builtin_amdgcn_perm(RE, RO, 0x07060100u);   // (V5, V6)
    const uint32_t P6 = __builtin_amdgcn_perm(RO, RE, 0x07060302u);   // (V6, V7)
    // the sum of one pixel on the v_dot2 accumulator chain, the rounding constant as its seed:
    // s = 2^15 + sum k V < 2^24, so the result (s >> 16) is byte 2 of s
    auto hz = [seed](uint32_t pa, uint32_t pb, uint32_t pc, uint32_t pd) {
      uint32_t s = dot2_acc(pd, 0x00000012u, seed);  // 18 V(j+3) + 2^15
      s = dot2_acc(pc, 0x00220031u, s);                // 49 V(j+1) + 34 V(j+2)
      s = dot2_acc(pb, 0x00360031u, s);                // 49 V(j-1) + 54 V(j)
      return dot2_acc(pa, 0x00220012u, s);             // 18 V(j-3) + 34 V(j-2)
    };
    const uint32_t s0 = hz(Pm3, Pm1, P1, P3), s1 = hz(Pm2, P0, P2, P4), s2 = hz(Pm1, P1, P3, P5),
                   s3 = hz(P0, P2, P4, P6);
    // bytes 2 of s0..s3 -> bytes 0..3 of r
    const uint32_t r = __builtin_amdgcn_perm(__builtin_amdgcn_perm(s3, s2, 0x0c0c0602u),
                                             __builtin_amdgcn_perm(s1, s0, 0x0c0c0602u), 0x05040100u);
    if (out) __builtin_amdgcn_raw_buffer_store_b32(r, ws, wo, (i - 6) * pitch, 0);  // row offset in an SGPR
  }
}

// ---------------------------------------------------------------------------------------------
// k_describe: one wavefront per surviving keypoint. IC_Angle (:75-102) sums the integer moments of
// the 749-pixel circle straight from the level (L1/L2 hits); the 256 steered tests (:105-151) read
// the blurred level; bits land as 4 wave ballots (64 pairs each = 8 descriptor bytes).
// k_describe's table: the 256 test pairs as floats (x0, y0, x1, y1)
__constant__ float4 c_patf[256];

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int group16_sum(int v) {  // sum over the 16-lane group of this lane
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
  return v;
}

// computeOrbDescriptor's cos / sin of the steering angle (ORBextractor.cc:109-110). With `using
// namespace std` (:66) `cos(angle)` on a float is std::cos(float) = glibc cosf / sinf, which are
// not correctly rounded ((float)cos((double)x) differs on 0.13 % of the reachable angles), so this
// is a port of glibc 2.35's sinf / cosf for |x| < 120 (sysdeps/ieee754/flt-32, the FMA ifunc
// variant x86-64 CPUs with FMA run): double polynomials on __sincosf_table with the same fma /
// multiply sequence. test_gpu_trig.py checks it against glibc on every float degree in [0, 360).
__device__ __forceinline__ double glibc_cos_poly(double x2) {
  const double x4 = x2 * x2;
  const double c1 = fma(x2, -0x1.ffffffd0c621cp-2, 1.0);
  const double c2 = fma(x2, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);
  const double x6 = x2 * x4;
  const double c = fma(x4, 0x1.55553e1068f19p-5, c1);
  return fma(c2, x6, c);
}
__device__ __forceinline__ double glibc_sin_poly(double x, double x2) {
  const double s1 = fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
  const double x3 = x2 * x;
  const double x5 = x3 * x2;
  const double s = fma(x3, -0x1.555545995a603p-3, x);
  return fma(s1, x5, s);
}
__device__ __forceinline__ void steer_cos_sin(float angle_deg, float factor_pi, float& c, float& s) {
  const float y = angle_deg * factor_pi;  // 0 <= y < 2 pi
  const uint32_t top12 = (__float_as_uint(y) >> 20) & 0x7ffu;
  const double x = (double)y;
  if (top12 <= 0x3f3u) {  // y < 0.75: no reduction; y < 2^-12: cosf = 1, sinf = y
    const double x2 = x * x;
    c = top12 <= 0x397u ? 1.0f : (float)glibc_cos_poly(x2);
    s = top12 <= 0x397u ? y : (float)glibc_sin_poly(x, x2);
    return;
  }
  const int n = ((int)(x * 0x1.45f306dc9c883p+23) + 0x800000) >> 24;  // reduce_fast
  const double r = fma(-(double)n, 0x1.921fb54442d18p+0, x);
  const double r2 = r * r;
  const double sp = glibc_sin_poly((n & 3) == 1 || (n & 3) == 2 ? -r : r, r2);  // r * sign[n & 3]
  const double cp = (n & 2) ? -glibc_cos_poly(r2) : glibc_cos_poly(r2);  // table 1 negates c0..c4
  // cosf: sin branch for odd n; sinf: sin branch for even n
  c = (float)((n & 1) ? sp : cp);
  s = (float)((n & 1) ? cp : sp);
}

// orbfe_debug_steer_trig: steer_cos_sin for the float degree values bits0 .. bits0 + n - 1
__global__ __launch_bounds__(256) void k_steer_trig(uint32_t bits0, uint32_t n, float factor_pi, float* c,
                                                     float* s) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  float cv, sv;
  steer_cos_sin(__uint_as_float(bits0 + i), factor_pi, cv, sv);
  c[i] = cv;
  s[i] = sv;
}

// Four keypoints per wavefront, 16 lanes each, so the per-keypoint scalar work (level lookup,
// fastAtan2, the cos/sin of computeOrbDescriptor) is shared by 4 keypoints. A wavefront issues all
// of its global loads before their first use (the IC_Angle window as 12-byte pieces, the blurred
// window as 8-byte pieces); the test pattern is copied to LDS once per block and the circle masks
// are computed, so the moments and the 256 tests read no global memory.
struct DwX3 {
  uint32_t x, y, z;
};

constexpr int DESC_WPB = 4;  // k_describe wavefronts per workgroup (4 keypoints each)
constexpr int DESC_THREADS = 64 * DESC_WPB;
// umax[0..15] (ORBextractor.cc:82-98; each <= 15) as 4-bit fields of two dwords: IC_Angle's
// circle masks are computed per dword, not looked up (a 4.4 KiB mask table in LDS left k_describe
// at 32 KiB per workgroup, two beside a DistributeOctTree block; 27 KiB without it: 84.0k vs
// 82.8k)
__constant__ uint32_t c_umax4[2];
__global__ __launch_bounds__(DESC_THREADS) void k_describe(ExtractArgs a) {
  __shared__ float4 s_pat[256];
  __shared__ __attribute__((aligned(16))) uint32_t s_win[4 * DESC_WPB][37 * 10];
  for (int k = threadIdx.x; k < 256; k += DESC_THREADS) s_pat[k] = c_patf[k];
  __syncthreads();  // before any wavefront may leave
  const int w = wave_id(), lane = lane_id(), grp = lane >> 4, l16 = lane & 15;
  const int2 blk = xcd_block2d();
  const int img = blk.y;
  const int slot = (blk.x * DESC_WPB + w) * 4 + grp;
  const int32_t* lc = a.lvlcnt + (long long)img * a.nlevels;
  if (blk.x == 0 && threadIdx.x == 0) {
    int tot = 0;
    for (int l = 0; l < a.nlevels; l++) tot += lc[l];
    a.out_counts[img] = tot;
  }
  bool valid = slot < a.total_key_slots;
  int l = 0;
  while (l + 1 < a.nlevels && slot >= a.levels[l + 1].key_begin) l++;
  const LevelDesc ld = a.levels[l];
  const int idx = slot - ld.key_begin;
  valid = valid && idx < lc[l];
  if (__ballot(valid) == 0) return;  // the whole wavefront is past the level ends
  int obase = idx;
  for (int k = 0; k < l; k++) obase += lc[k];
  const uint32_t key = valid ? a.lvlkeys[(long long)img * a.lvlkey_stride + slot] : pack_key(19, 19, 0);
  // (an invalid group reads a harmless in-range window of the same level and writes nothing)
  const int cx = key_x(key), cy = key_y(key), score = key_s(key);
  // keypoints lie in [19, w-20] x [19, h-20] (FAST never fires within 3 px of a cell ROI whose
  // origin is minBorder - 3 = 16), so both windows below stay inside the padded rows
  const long long lbase = (long long)img * a.pyr_stride + ld.pyr_off;
  const int pitch = ld.pitch;
  // 1. every global load in flight at once. IC_Angle window: rows cy-15..cy+15, 9 dwords per row
  //    from xa = (cx-15) & ~3, as three 12-byte pieces; piece i = l16 + 16 k lies in row i / 3,
  //    16 rows further every 3 k. Blurred window: rows cy-18..cy+18, 10 dwords from
  //    xb = (cx-18) & ~3, as five 8-byte pieces (row i / 5, 16 rows further every 5 k).
  const int xa = (cx - 15) & ~3, xb = (cx - 18) & ~3;
  const uint8_t* usrc = a.pyr + lbase + (long long)(cy - 15) * pitch + xa;
  const uint8_t* bsrc = a.blur + lbase + (long long)(cy - 18) * pitch + xb;
  const int step16 = 16 * pitch;
  int ur[3], uc[3], br[5], bc[5];
#pragma unroll
  for (int q = 0; q < 3; q++) {
    ur[q] = (l16 + 16 * q) / 3;
    uc[q] = l16 + 16 * q - 3 * ur[q];
  }
#pragma unroll
  for (int q = 0; q < 5; q++) {
    br[q] = (l16 + 16 * q) / 5;
    bc[q] = l16 + 16 * q - 5 * br[q];
  }
  DwX3 mu[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    mu[k] = DwX3{0u, 0u, 0u};
    if (l16 + 16 * k < 93) __builtin_memcpy(&mu[k], usrc + (k / 3) * step16 + ur[k % 3] * pitch + 12 * uc[k % 3], 12);
  }
  uint2 bw[12];
#pragma unroll
  for (int k = 0; k < 12; k++) {
    bw[k] = make_uint2(0u, 0u);
    if (l16 + 16 * k < 185) __builtin_memcpy(&bw[k], bsrc + (k / 5) * step16 + br[k % 5] * pitch + 8 * bc[k % 5], 8);
  }
  // 2. IC_Angle moments (:75-102) over the 749-pixel circle: bytes with |u| <= umax[|v|] (a byte
  //    mask per dword from umax), sums of I and col * I by byte dot products
  const int msh = (cx - 15) & 3;
  const uint32_t um_lo = c_umax4[0], um_hi = c_umax4[1];
  int m01 = 0, m10 = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    if (l16 + 16 * k < 93) {
      const int r = ur[k % 3] + 16 * (k / 3), v = r - 15;
      const uint32_t d3[3] = {mu[k].x, mu[k].y, mu[k].z};
      const int av = v < 0 ? -v : v;
      const int um = (int)(((av < 8 ? um_lo : um_hi) >> (4 * (av & 7))) & 15u);
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const int c = 3 * uc[k % 3] + d;  // dword of the row
        // bytes b of dword c with |u| <= um, u = -15 - msh + 4 c + b
        const int blo = min(max(15 + msh - 4 * c - um, 0), 4), bhi = min(max(16 + msh - 4 * c + um, 0), 4);
        const uint32_t msk = blo < bhi ? (uint32_t)((((1ull << (8 * (bhi - blo))) - 1ull)) << (8 * blo)) : 0u;
        const uint32_t px = d3[d] & msk;
        const int sI = (int)__builtin_amdgcn_udot4(px, 0x01010101u, 0u, false);
        const int sC = (int)__builtin_amdgcn_udot4(px, (uint32_t)(4 * c) * 0x01010101u + 0x03020100u, 0u, false);
        m10 += sC + (xa - cx) * sI;  // sum u I with u = xa + col - cx
        m01 += v * sI;
      }
    }
  }
  m01 = group16_sum(m01);
  m10 = group16_sum(m10);
  // the blurred pieces -> LDS (rows of 40 bytes), ahead of the angle arithmetic
  uint8_t* winb = reinterpret_cast<uint8_t*>(s_win[w * 4 + grp]);
#pragma unroll
  for (int k = 0; k < 12; k++)
    if (l16 + 16 * k < 185)
      *reinterpret_cast<uint2*>(winb + (br[k % 5] + 16 * (k / 5)) * 40 + 8 * bc[k % 5]) = bw[k];
  const float angle = fast_atan2_dev((float)m01, (float)m10, a.atan);
  float ca, sb;
  steer_cos_sin(angle, a.factor_pi, ca, sb);
  wave_sync();
  // 3. the 256 steered tests (:105-151) on the LDS window, pixel (dy, dx) at byte
  //    (dy + 18) * 40 + (dx + cx - xb); test p = 16 j + l16 lands in bit l16 of the group's
  //    16-bit slice of ballot j = descriptor bytes 2j, 2j+1
  const uint8_t* wb = winb + 18 * 40 + (cx - xb);
  uint32_t dv = 0;  // lane l16 < 8 collects descriptor dword l16 = bytes 4 l16 .. 4 l16 + 3
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int p = 16 * j + l16;
    // row = cvRound(x sin + y cos), col = cvRound(x cos - y sin) (:115-117): the products and the
    // sum in packed fp32 (separately rounded, as the reference), cvRound's half-even by adding
    // 1.5 * 2^23 and reading the integer out of the mantissa
    const float4 P = s_pat[p];
    const f32x2 sc = {sb, ca}, cs = {ca, -sb}, magic = {12582912.0f, 12582912.0f};
    const f32x2 q0 = (f32x2){P.x, P.x} * sc + (f32x2){P.y, P.y} * cs + magic;
    const f32x2 q1 = (f32x2){P.z, P.z} * sc + (f32x2){P.w, P.w} * cs + magic;
    // the bits of q are 0x4B400000 + v (|v| < 2^22): their low 24 bits 0x400000 + v feed a
    // full-rate v_mad_u32_u24 (a plain 32-bit multiply-add here compiles to quarter-rate
    // v_mad_u64_u32); (0x400000 + vr) * 40 + 0x4B400000 + vc - 0x55400000 = 40 vr + vc
    const int i0 = (int)(__umul24((uint32_t)__float_as_int(q0.x), 40u) + (uint32_t)__float_as_int(q0.y) - 0x55400000u);
    const int i1 = (int)(__umul24((uint32_t)__float_as_int(q1.x), 40u) + (uint32_t)__float_as_int(q1.y) - 0x55400000u);
    const int t0 = wb[i0];
    const int t1 = wb[i1];
    const uint32_t hv = (uint32_t)(wave_ballot(t0 < t1) >> (16 * grp)) & 0xffffu;
    if (l16 == (j >> 1)) dv |= hv << (16 * (j & 1));
  }
  if (!valid) return;
  const long long o = (long long)img * a.out_cap + obase;
  if (l16 < 8) reinterpret_cast<uint32_t*>(a.out_desc + o * 32)[l16] = dv;
  if (l16 == 0) {
    orbfe_keypoint kp;
    kp.x = (float)cx;
    kp.y = (float)cy;
    if (l != 0) {
      kp.x *= ld.scale;
      kp.y *= ld.scale;
    }
    kp.size = (float)ld.size;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    a.out_kps[o] = kp;
  }
}

// =============================================================================================
// host side
namespace {

inline int h_round(float v) { return (int)std::lrintf(v); }
inline int h_floor(float v) { int i = (int)v; return i - (i > v); }
inline short h_sat_short(float v) {
  int i = h_round(v);
  return (short)std::min(std::max(i, -32768), 32767);
}
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

// Fork/join events between the extractor's two streams order device work only (nothing on the
// host waits on them), so they skip the system-scope fence: without it the record + wait pair
// costs less queue time between the dependent launches.
static const unsigned kForkJoinEvent = hipEventDisableTiming | hipEventDisableSystemFence;

// Host worker pool of a handle (the host-buffer entry points' staging copies): parallel_for runs
// f(0..n-1) on the workers and the calling thread and returns when all are done.
class HostPool {
 public:
  explicit HostPool(int workers) {
    for (int i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void parallel_for(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
      for (int i = 0; i < n; i++) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      n_ = n;
      next_.store(0);
      left_ = n;
      gen_++;
    }
    cv_.notify_all();
    run();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void run() {
    int done = 0;
    for (int i; (i = next_.fetch_add(1)) < n_;) {
      (*job_)(i);
      done++;
    }
    if (done) {
      std::lock_guard<std::mutex> g(m_);
      left_ -= done;
      if (left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    unsigned long long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || (gen_ != seen && job_ != nullptr); });
        if (stop_) return;
        seen = gen_;
      }
      run();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0, left_ = 0;
  std::atomic<int> next_{0};
  unsigned long long gen_ = 0;
  bool stop_ = false;
};

// k_octree's LDS plan for a range of levels: node arena, scan and sort capacities from those levels'
// budgets and cell counts, and as many keys (two ping-pong halves) as the budget leaves
struct OctPlan {
  int node_cap = 0, sort_cap = 0, scan_cap = 0, key_lds_cap = 0;
  size_t lds = 0;
};

constexpr int OCT_LDS_KB = 80;  // k_octree's LDS per workgroup (two per CU)

struct orbfe_extractor {
  int device = 0;
  int nfeatures, nlevels, ini_th, min_th;
  double scale_factor;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> nfeat;
  int umax[16];
  int resize_mode = ORBFE_RESIZE_SIMD128;
  int octree_key_cap_override = -1;  // orbfe_debug_set_octree_key_cap
  int fast_side_levels = -1;         // orbfe_debug_set_fast_side_levels (-1: the default, 3 levels)
  int inline_side = 0;               // orbfe_debug_set_inline_side: side-stream work on the launch stream
  hipStream_t side_ext = nullptr;    // orbfe_set_side_stream: a caller's stream instead of h->side
  int blur_mode = 0;                 // orbfe_debug_set_blur_mode
  int octree_split = 5;              // orbfe_debug_set_octree_split: levels 0..k-1 and k..L-1 in two launches
                                     // (k = 5 86.7-86.9k vs 4 85.7-85.9k stereo frames/s, round 6)
  int lat_sched = 1;                 // orbfe_debug_set_latency_schedule: levels on the side (< 8 images)
  // Calls of fewer than 8 images choose per image count between the latency schedule on two streams
  // and the same sequence on the launch stream alone, by timing their first host-buffer calls:
  // when the runtime has put the handle's launch and side streams on one hardware queue (its pool
  // holds GPU_MAX_HW_QUEUES queues, 4 by default, for all the process's streams), the cross-stream
  // waits cost ~140 us per call -- one KITTI image 0.275-0.283 ms with 4+ idle handles alive vs
  // 0.183 on one stream and 0.130-0.135 on two distinct queues (profiles/r6_c2_queues.txt).
  // orbfe_debug_set_schedule_autotune(h, 0) (or ORBFE_SCHED_AUTOTUNE=0): always two streams.
  struct SchedTune {
    int calls = 0, decided = -1;  // decided: -1 still timing, 0 two streams, 1 the launch stream
    std::vector<double> t_two, t_one;
  } tune[8];
  int autotune = 1;
  bool call_inline = false;          // this call's choice (launch_extract)
  int oct_threads_small = 512;       // k_octree block size for calls of < 8 images (orbfe_debug_set_octree_threads)
  int oct_threads_batch = 256;       // ... and for batches of 8+
  int oct_threads_l0 = 0;            // ... for a small call's launch that holds level 0 (0: oct_threads_small)
  int oct_small_small = OCT_SMALL;   // k_octree's thread-serial node size for calls of < 8 images ...
  int oct_small_batch = OCT_SMALL;   // ... and batches (orbfe_debug_set_octree_serial)
  int oct_hi_kb = OCT_LDS_KB, oct_lo_kb = OCT_LDS_KB / 2;  // their LDS budgets (orbfe_debug_set_octree_lds)
  bool device_call = false;          // the current call is orbfe_extract_batch_device (may take the split)
  int fast_wpb_side = 4, fast_wpb_main = 1;  // k_fast cells per workgroup (orbfe_debug_set_fast_wpb)
  int fast_side_merge = 0;           // orbfe_debug_set_fast_side_merge: side FAST levels 1..k-1 in one launch
  // k_pyramid tiles per image (x, y) for calls of < 8 images / batches; 0: the per-level resize
  // chain (orbfe_debug_set_pyramid_tiles). One KITTI image: orbfe_extract p50 0.160 ms at 16 x 12
  // vs 0.169 through the chain (32 x 24 0.163, 8 x 6 0.163; profiles/r6_c2_pyramid.txt); batches
  // keep the chain: its launches fill the chip, the tiles' level-by-level latency chains do not
  // (C3 bench 43-59k vs 86.9k stereo frames/s, profiles/r6_sweep_pyramid.txt)
  int pyr_tiles_small[2] = {16, 12}, pyr_tiles_batch[2] = {0, 0};
  struct PyrPlan {
    int ntiles = 0, half_dw = 0;
    size_t lds = 0;
    PyrTileLevel* d_tiles = nullptr;
  } pyr_small, pyr_batch;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;               // k_blur runs here, beside k_fast + k_octree
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_l0 = nullptr, ev_f0 = nullptr;
  hipEvent_t ev_pyr = nullptr;              // pyramid complete (orbfe_extractor_pyramid_event)
  std::vector<hipEvent_t> ev_lvl;           // level l built (per-level FAST on the side stream)
  // geometry
  int rows = -1, cols = -1, geom_mode = -1;
  std::vector<LevelDesc> levels;
  std::vector<CellDesc> cells;
  std::vector<int2> xtab, ytab;
  long long pyr_stride = 0, cand_stride = 0, keyscr_stride = 0, lvlkey_stride = 0;
  int total_key_slots = 0, roi_w_max = 0, roi_h_max = 0, node_cap = 0, sort_cap = 0, blur_tiles = 0;
  int scan_cap = 0, key_lds_cap = 0;
  OctPlan oct_all, oct_hi, oct_lo;  // k_octree LDS plans: one launch, or levels [0, split) / [split, L)
  LevelDesc* d_levels = nullptr;
  CellDesc* d_cells = nullptr;
  int2* d_xtab = nullptr;
  int2* d_ytab = nullptr;
  int4* d_ywin = nullptr;
  uint4* d_rgrp = nullptr;
  int* d_rgx0 = nullptr;
  // batch buffers
  int batch_cap = 0;
  uint8_t* d_in = nullptr;
  size_t in_bytes = 0;
  uint8_t* d_pyr = nullptr;
  uint8_t* d_blur = nullptr;
  uint32_t* d_cand = nullptr;
  int32_t* d_cellcnt = nullptr;
  uint32_t* d_keys_a = nullptr;
  uint32_t* d_keys_b = nullptr;
  uint32_t* d_lvlkeys = nullptr;
  int32_t* d_lvlcnt = nullptr;
  // host-buffer entry points' results: one block [slots x keypoint][slots x 32 B][images x count],
  // laid out like its pinned host mirror h_out, so a small call's results go down in one copy
  uint8_t* d_out = nullptr;
  orbfe_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  int32_t* d_counts = nullptr;
  size_t out_cap_alloc = 0;  // keypoint slots (a multiple of 64)
  int out_n_alloc = 0;       // image counts
  size_t out_bytes = 0;
  // host-buffer entry points: worker pool for the staging copies, copy streams and per-chunk
  // events of the H2D / extract / D2H pipeline
  HostPool* pool = nullptr;
  hipStream_t h2d = nullptr, d2h = nullptr;
  std::vector<hipEvent_t> ev_in, ev_ext, ev_out;
  // pinned staging of the host-buffer entry points
  uint8_t* h_in = nullptr;
  uint8_t* h_in_dev = nullptr;  // h_in as the device addresses it (k_copy0 reads it over PCIe)
  size_t h_in_bytes = 0;
  // calls of < 8 images: k_copy0 reads the staged images straight from pinned host memory instead
  // of after a separate H2D copy (orbfe_debug_set_zero_copy)
  int zc_in = 1;
  bool input_l0 = false;  // this call's input is already in the level-0 layout (k_copy_l0)
  // ... and k_octree / k_describe write the results straight into the pinned mirror h_out instead
  // of a device block copied down afterwards (plain calls: no hook reads the device outputs)
  int zc_out = 1;
  uint8_t* h_out_dev = nullptr;
  uint8_t* h_out = nullptr;
  size_t h_out_bytes = 0;
  // last call (for get_level)
  const uint8_t* last_img0 = nullptr;
  long long last_img_stride = 0;
  int last_img_pitch = 0, last_n = 0;
  hipStream_t last_stream = nullptr;  // the stream the last call's pyramids were built on
  // mvImagePyramid on the host (orbfe_get_level): one pinned block holding every image of the last
  // call at the device layout (levels packed, rows `pitch` apart), so all levels of all images stay
  // valid together until the next extract call. An image is copied on its first access, or during
  // the extraction itself when the handle prefetches (orbfe_extractor_set_host_pyramid).
  unsigned long long gen = 0;            // extract calls so far (the block's validity)
  uint8_t* h_pyr = nullptr;
  size_t h_pyr_bytes = 0;
  std::vector<unsigned long long> h_pyr_gen;  // per image: the call whose pyramid the block holds
  int host_pyramid = 0;                  // prefetch the pyramids to h_pyr in the host-buffer calls
  hipEvent_t ev_hpyr = nullptr;          // the prefetch copies are done
  bool hpyr_pending = false;
  // Frame::ComputeStereoMatches scratch (orbfe_stereo.hip)
  OrbfeStereoScratch* stereo = nullptr;
  // launch_extract's enqueue sequence captured once per distinct set of arguments and replayed as
  // a hipGraph (orbfe_extractor_set_graphs; `graphs` keyed by everything the sequence depends on).
  // Off by default: measured slower on MI355X / ROCm 7.2
  int use_graphs = 0;
  struct GraphEntry {
    std::vector<uintptr_t> key;
    hipGraphExec_t exec;
    unsigned long long used;
  };
  std::vector<GraphEntry> graphs;
  unsigned long long graph_clock = 0;
  unsigned long long graph_hits = 0, graph_captures = 0;
};

static OctPlan octree_plan(const std::vector<LevelDesc>& lv, int l0, int l1, int budget_kb, int key_cap_override);
static size_t octree_lds(const orbfe_extractor* h);

// k_pyramid's tiles: level l's 4-column groups and rows cut into tx x ty owned blocks; from the top
// level down, each tile's computed region at level l is its owned block joined with what its
// computed region at level l + 1 reads (rows clamp(sy), clamp(sy + 1); the 8-byte window from
// rgx0, cut at the level's last column). Entry 0 holds level 0's footprint (read from the pyramid
// block, not computed). Returns the LDS dwords one level buffer needs (0: no plan -- a level
// without the 8-byte window, one level, or a tile past the LDS budget).
static int pyramid_plan(const std::vector<LevelDesc>& lv, const std::vector<int2>& yt, const std::vector<int>& rgx0,
                        int tx, int ty, std::vector<PyrTileLevel>& out, int& tab_dw) {
  const int L = (int)lv.size();
  out.clear();
  tab_dw = 0;
  if (L < 2 || L > PYR_MAX_LEVELS || tx <= 0 || ty <= 0) return 0;
  for (int l = 1; l < L; l++)
    if (!lv[l].rwin_ok) return 0;
  int half = 0, tab = 0;
  for (int i = 0; i < ty; i++)
    for (int j = 0; j < tx; j++) {
      std::vector<PyrTileLevel> T(L);
      int fg_a = 0, fg_b = 0, fy_a = 0, fy_b = 0;  // footprint in the level below (empty)
      for (int l = L - 1; l >= 0; l--) {
        PyrTileLevel& t = T[l];
        std::memset(&t, 0, sizeof(t));
        int ga = fg_a, gb = fg_b, ya = fy_a, yb = fy_b;
        if (l >= 1) {
          const int G = (lv[l].w + 3) / 4, H = lv[l].h;
          t.og_a = (int16_t)(j * G / tx);
          t.og_b = (int16_t)((j + 1) * G / tx);
          t.oy_a = (int16_t)(i * H / ty);
          t.oy_b = (int16_t)((i + 1) * H / ty);
          if (t.og_a < t.og_b && t.oy_a < t.oy_b) {
            if (ga < gb && ya < yb) {
              ga = std::min(ga, (int)t.og_a);
              gb = std::max(gb, (int)t.og_b);
              ya = std::min(ya, (int)t.oy_a);
              yb = std::max(yb, (int)t.oy_b);
            } else {
              ga = t.og_a, gb = t.og_b, ya = t.oy_a, yb = t.oy_b;
            }
          }
        }
        t.ng_a = (int16_t)ga;
        t.ng_b = (int16_t)gb;
        t.ny_a = (int16_t)ya;
        t.ny_b = (int16_t)yb;
        const int ng = gb - ga;
        t.gmagic = ng > 0 ? (uint32_t)((0x100000000ull + 4 * ng - 1) / (4 * ng)) : 0u;  // items / (4 ng) columns
        if (ga >= gb || ya >= yb) t.ng_a = t.ng_b = t.ny_a = t.ny_b = 0;  // nothing computed
        if (l >= 1 && l + 1 < L && ga < gb && ya < yb) half = std::max(half, (ng + 3) * (yb - ya));
        fg_a = fg_b = fy_a = fy_b = 0;
        if (l >= 1 && ga < gb && ya < yb) {  // what this computed region reads of level l - 1
          const LevelDesc& d = lv[l];
          const LevelDesc& s = lv[l - 1];
          fy_a = std::min(std::max(yt[d.tab_y + ya].x, 0), s.h - 1);
          fy_b = std::min(std::max(yt[d.tab_y + yb - 1].x + 1, 0), s.h - 1) + 1;
          fg_a = rgx0[d.rgrp_begin + ga] >> 2;
          fg_b = (std::min(rgx0[d.rgrp_begin + gb - 1] + 7, s.w - 1) >> 2) + 1;
        }
      }
      int off = 0;  // the staged tables, levels 1..L-1
      for (int l = 1; l < L; l++) {
        T[l].tab_off = off;
        off += 9 * (T[l].ng_b - T[l].ng_a) + 2 * (T[l].ny_b - T[l].ny_a);
      }
      tab = std::max(tab, off);
      out.insert(out.end(), T.begin(), T.end());
    }
  half = std::max(half, 1);
  tab_dw = tab;
  if ((2 * (size_t)half + tab) * 4 > 64 * 1024) {
    out.clear();
    return 0;
  }
  return half;
}
static void drop_graphs(orbfe_extractor* h);
static int compute_geometry(orbfe_extractor* h, int rows, int cols) {
  if (h->rows == rows && h->cols == cols && h->geom_mode == h->resize_mode) return ORBFE_OK;
  const int L = h->nlevels;
  std::vector<LevelDesc> lv(L);
  std::vector<CellDesc> cells;
  std::vector<int2> xt, yt;
  std::vector<int4> yw;  // k_resize_win row table, indexed like yt
  std::vector<uint4> rgrp;
  std::vector<int> rgx0;
  long long pyr = 0;
  int cand = 0, keys = 0, rwmax = 0, rhmax = 0, ncap = 0, tiles = 0;
  for (int l = 0; l < L; l++) {
    LevelDesc& d = lv[l];
    std::memset(&d, 0, sizeof(d));
    d.w = h_round((float)cols * h->inv_scale[l]);
    d.h = h_round((float)rows * h->inv_scale[l]);
    if (d.w > 4095 || d.h > 4095)  // candidate / survivor keys hold x and y in 12 bits each
      return orbfe_set_error(ORBFE_ERR_ARG, "image too large: width and height must be below 4096");
    const int minB = 16, maxBX = d.w - 16, maxBY = d.h - 16;  // EDGE_THRESHOLD - 3
    const int bw = maxBX - minB, bh = maxBY - minB;
    if (bw < 30 || bh < 30)
      return orbfe_set_error(ORBFE_ERR_ARG, "image too small for the pyramid: a level has < 62 px");
    d.nini = (int)std::round((float)bw / bh);
    if (d.nini < 1 || d.nini > 64)
      return orbfe_set_error(ORBFE_ERR_ARG, "unsupported aspect ratio (DistributeOctTree nIni)");
    d.hx = (float)bw / d.nini;
    // initial node of a key = (int)(x / hX) (:575) as compares against host thresholds (the key
    // x are integers in [0, bw]; the same IEEE float division as the reference)
    for (int b = 0; b < 8; b++) {
      int x = 0;
      while (x <= bw + 1 && (int)((float)x / d.hx) < b) x++;
      d.ini_thr[b] = x;
    }
    d.rel_w = bw;
    d.rel_h = bh;
    d.budget = h->nfeat[l];
    d.scale = h->scale[l];
    d.size = (int)(31 * h->scale[l]);
    // rows carry 4 bytes of left and >= 8 of right padding holding REFLECT_101 columns
    // (-3..-1 and w..w+2, written by k_copy0 / k_resize) so k_blur reads aligned dwords only
    d.pitch = (int)align_up(d.w + 4 + 8, 64);
    d.pyr_off = pyr + 4;  // column 0 of row 0
    pyr += (long long)d.pitch * d.h;
    // cells (:776-832)
    const float width = (float)bw, height = (float)bh;
    const int nColsC = (int)(width / 30.f), nRowsC = (int)(height / 30.f);
    const int wCell = (int)std::ceil(width / nColsC), hCell = (int)std::ceil(height / nRowsC);
    d.cell_begin = (int)cells.size();
    d.cand_begin = cand;
    for (int i = 0; i < nRowsC; i++) {
      const float iniY = (float)(minB + i * hCell);
      float maxY = iniY + hCell + 6;
      if (iniY >= maxBY - 3) continue;
      if (maxY > maxBY) maxY = (float)maxBY;
      for (int j = 0; j < nColsC; j++) {
        const float iniX = (float)(minB + j * wCell);
        float maxX = iniX + wCell + 6;
        if (iniX >= maxBX - 6) continue;
        if (maxX > maxBX) maxX = (float)maxBX;
        CellDesc c;
        std::memset(&c, 0, sizeof(c));
        c.level = (int16_t)l;
        c.x0 = (int16_t)(int)iniX;
        c.y0 = (int16_t)(int)iniY;
        c.rw = (int16_t)((int)maxX - (int)iniX);
        c.rh = (int16_t)((int)maxY - (int)iniY);
        c.ox = (int16_t)(j * wCell);
        c.oy = (int16_t)(i * hCell);
        const int dw = c.rw - 6, dh = c.rh - 6;
        c.cap = (dw > 0 && dh > 0) ? ((dw + 1) / 2) * ((dh + 1) / 2) : 0;
        c.slot = cand;
        c.pyr_off = (int32_t)d.pyr_off;
        c.pitch = d.pitch;
        cand += c.cap;
        rwmax = std::max(rwmax, (int)c.rw);
        rhmax = std::max(rhmax, (int)c.rh);
        cells.push_back(c);
      }
    }
    d.ncells = (int)cells.size() - d.cell_begin;
    d.cand_cap = cand - d.cand_begin;
    {  // k_blur strips of BS_W x BS_H, the remainder columns in bands of blur_h x BS_H rows
      d.tiles_x = d.w / BS_W;
      const int rem = d.w - d.tiles_x * BS_W;
      d.blur_h = rem == 0 ? 0 : rem <= 14 * 4 ? 4 : rem <= 30 * 4 ? 2 : 1;
      d.tile_begin = tiles;
      tiles += d.tiles_x * ((d.h + BS_H - 1) / BS_H) + (d.blur_h ? (d.h + BS_H * d.blur_h - 1) / (BS_H * d.blur_h) : 0);
    }
    d.key_begin = keys;
    d.key_cap = std::max(d.budget + 3, 4 * d.nini);
    keys += d.key_cap;
    ncap = std::max(ncap, d.key_cap + 4);
    // resize tables (OpenCV resize(), INTER_LINEAR, fixed point)
    if (l > 0) {
      const LevelDesc& s = lv[l - 1];
      const double inv_sx = (double)d.w / s.w, inv_sy = (double)d.h / s.h;
      const double scx = 1. / inv_sx, scy = 1. / inv_sy;
      d.tab_x = (int)xt.size();
      d.tab_y = (int)yt.size();
      int xmax = d.w;
      for (int dx = 0; dx < d.w; dx++) {
        float fx = (float)((dx + 0.5) * scx - 0.5);
        int sx = h_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= s.w) {
          xmax = std::min(xmax, dx);
          if (sx >= s.w - 1) { fx = 0.f; sx = s.w - 1; }
        }
        const short a0 = h_sat_short((1.f - fx) * 2048.f), a1 = h_sat_short(fx * 2048.f);
        xt.push_back(make_int2(sx, (int)(((unsigned)(unsigned short)a1 << 16) | (unsigned short)a0)));
      }
      for (int dy = 0; dy < d.h; dy++) {
        float fy = (float)((dy + 0.5) * scy - 0.5);
        int sy = h_floor(fy);
        fy -= sy;
        const short b0 = h_sat_short((1.f - fy) * 2048.f), b1 = h_sat_short(fy * 2048.f);
        yt.push_back(make_int2(sy, (int)(((unsigned)(unsigned short)b1 << 16) | (unsigned short)b0)));
        const int r0 = std::min(std::max(sy, 0), s.h - 1), r1 = std::min(std::max(sy + 1, 0), s.h - 1);
        yw.push_back(make_int4(r0 * (s.pitch / 4), r1 * (s.pitch / 4), yt.back().y, 0));
      }
      d.xmax = xmax;
      // 4-column groups: the taps of output columns 4g..4g+3 as byte selectors into the 8-byte
      // source window starting at sx(4g); columns at or past xmax take (sx, sx) with alpha
      // (2048, 0), i.e. S[sx] * ONE as OpenCV does there
      d.rgrp_begin = (int)rgx0.size();
      d.rwin_ok = 1;
      for (int g = 0; 4 * g < d.w; g++) {
        const int x0 = xt[d.tab_x + 4 * g].x;
        uint32_t sel[4], alp[4];
        for (int k = 0; k < 4; k++) {
          const int col = std::min(4 * g + k, d.w - 1);
          const int2 e = xt[d.tab_x + col];
          const int o = e.x - x0;
          if (col >= xmax) {
            sel[k] = (uint32_t)o | 0x0c00u | ((uint32_t)o << 16) | 0x0c000000u;
            alp[k] = 16u * 2048u;
          } else {
            sel[k] = (uint32_t)o | 0x0c00u | ((uint32_t)(o + 1) << 16) | 0x0c000000u;
            alp[k] = 16u * (uint32_t)e.y;  // x 16: see resize_win_row (each u16 half <= 32768)
          }
          if (o < 0 || o + 1 > 7) d.rwin_ok = 0;
        }
        rgx0.push_back(x0);
        rgrp.push_back(make_uint4(sel[0], sel[1], sel[2], sel[3]));
        rgrp.push_back(make_uint4(alp[0], alp[1], alp[2], alp[3]));
      }
      int se = 0;
      if (h->resize_mode == ORBFE_RESIZE_SIMD128) {
        se = 16 * (d.w / 16);
        if (se < d.w - 8) se += 8;
      }
      d.simd_end = se;
    }
  }
  // release old geometry buffers and upload new ones (and the launch graphs that point at them)
  hipSetDevice(h->device);
  drop_graphs(h);
  hipFree(h->d_rgrp);
  hipFree(h->d_rgx0);
  h->d_rgrp = nullptr;
  h->d_rgx0 = nullptr;
  if (!rgx0.empty()) {
    ORBFE_HIP_CHECK(hipMalloc(&h->d_rgrp, sizeof(uint4) * rgrp.size()));
    ORBFE_HIP_CHECK(hipMalloc(&h->d_rgx0, sizeof(int) * rgx0.size()));
    ORBFE_HIP_CHECK(hipMemcpy(h->d_rgrp, rgrp.data(), sizeof(uint4) * rgrp.size(), hipMemcpyHostToDevice));
    ORBFE_HIP_CHECK(hipMemcpy(h->d_rgx0, rgx0.data(), sizeof(int) * rgx0.size(), hipMemcpyHostToDevice));
  }
  hipFree(h->d_levels);
  hipFree(h->d_cells);
  hipFree(h->d_xtab);
  hipFree(h->d_ytab);
  hipFree(h->d_ywin);
  h->d_levels = nullptr;
  h->d_cells = nullptr;
  h->d_xtab = h->d_ytab = nullptr;
  h->d_ywin = nullptr;
  ORBFE_HIP_CHECK(hipMalloc(&h->d_levels, sizeof(LevelDesc) * L));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_cells, sizeof(CellDesc) * std::max<size_t>(cells.size(), 1)));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_xtab, sizeof(int2) * std::max<size_t>(xt.size(), 1)));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_ytab, sizeof(int2) * std::max<size_t>(yt.size(), 1)));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_ywin, sizeof(int4) * std::max<size_t>(yw.size(), 1)));
  ORBFE_HIP_CHECK(hipMemcpy(h->d_levels, lv.data(), sizeof(LevelDesc) * L, hipMemcpyHostToDevice));
  if (!cells.empty())
    ORBFE_HIP_CHECK(hipMemcpy(h->d_cells, cells.data(), sizeof(CellDesc) * cells.size(), hipMemcpyHostToDevice));
  if (!xt.empty())
    ORBFE_HIP_CHECK(hipMemcpy(h->d_xtab, xt.data(), sizeof(int2) * xt.size(), hipMemcpyHostToDevice));
  if (!yt.empty())
    ORBFE_HIP_CHECK(hipMemcpy(h->d_ytab, yt.data(), sizeof(int2) * yt.size(), hipMemcpyHostToDevice));
  if (!yw.empty())
    ORBFE_HIP_CHECK(hipMemcpy(h->d_ywin, yw.data(), sizeof(int4) * yw.size(), hipMemcpyHostToDevice));
  h->levels = lv;
  h->cells = cells;
  h->xtab = xt;
  h->ytab = yt;
  h->pyr_stride = (long long)align_up((size_t)std::max<long long>(pyr, 64), 256);
  h->cand_stride = (long long)align_up((size_t)std::max(cand, 1), 64);
  h->keyscr_stride = h->cand_stride;
  h->lvlkey_stride = (long long)align_up((size_t)keys, 64);
  h->total_key_slots = keys;
  h->blur_tiles = tiles;
  h->roi_w_max = rwmax;
  h->roi_h_max = rhmax;
  h->oct_all = octree_plan(lv, 0, L, OCT_LDS_KB, h->octree_key_cap_override);
  // two launches: the large levels at the full budget (two blocks per CU), the small ones at half
  // of it (four per CU), so the short blocks of levels >= split hold half the LDS
  const int ks = std::min(std::max(h->octree_split, 0), L);
  h->oct_hi = octree_plan(lv, 0, ks, h->oct_hi_kb, h->octree_key_cap_override);
  h->oct_lo = octree_plan(lv, ks, L, h->oct_lo_kb, h->octree_key_cap_override);
  h->node_cap = h->oct_all.node_cap;
  h->sort_cap = h->oct_all.sort_cap;
  h->scan_cap = h->oct_all.scan_cap;
  h->key_lds_cap = h->oct_all.key_lds_cap;
  (void)ncap;
  for (int k = 0; k < 2; k++) {
    orbfe_extractor::PyrPlan& P = k == 0 ? h->pyr_small : h->pyr_batch;
    const int* tt = k == 0 ? h->pyr_tiles_small : h->pyr_tiles_batch;
    hipFree(P.d_tiles);
    P = orbfe_extractor::PyrPlan();
    std::vector<PyrTileLevel> tiles;
    int tab_dw = 0;
    const int half = pyramid_plan(lv, yt, rgx0, tt[0], tt[1], tiles, tab_dw);
    if (half > 0) {
      ORBFE_HIP_CHECK(hipMalloc(&P.d_tiles, sizeof(PyrTileLevel) * tiles.size()));
      ORBFE_HIP_CHECK(
          hipMemcpy(P.d_tiles, tiles.data(), sizeof(PyrTileLevel) * tiles.size(), hipMemcpyHostToDevice));
      P.ntiles = tt[0] * tt[1];
      P.half_dw = half;
      P.lds = sizeof(uint32_t) * (2 * (size_t)half + (size_t)tab_dw);
    }
  }
  h->rows = rows;
  h->cols = cols;
  h->geom_mode = h->resize_mode;
  h->batch_cap = 0;  // strides changed: reallocate batch buffers on the next call
  // k_octree's dynamic LDS limit, set here rather than per launch (a host call a captured launch
  // sequence cannot replay); the attribute is per function and device, so the largest plan any
  // handle of the process asked for on this device stays in force there
  constexpr int kMaxDevices = 64;
  static std::mutex attr_mu;
  static int attr_lds[kMaxDevices] = {};
  {
    std::lock_guard<std::mutex> lk(attr_mu);
    const int need = (int)std::max(h->oct_all.lds, std::max(h->oct_hi.lds, h->oct_lo.lds));
    int* have = h->device >= 0 && h->device < kMaxDevices ? &attr_lds[h->device] : nullptr;
    if (need <= 160 * 1024 && (!have || need > *have)) {
      ORBFE_HIP_CHECK(
          hipFuncSetAttribute((const void*)k_octree<256>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      ORBFE_HIP_CHECK(
          hipFuncSetAttribute((const void*)k_octree<512>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      ORBFE_HIP_CHECK(
          hipFuncSetAttribute((const void*)k_octree<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      if (have) *have = need;
    }
  }
  return ORBFE_OK;
}

static OctPlan octree_plan(const std::vector<LevelDesc>& lv, int l0, int l1, int budget_kb, int key_cap_override) {
  OctPlan p;
  if (l1 <= l0) return p;
  int ncap = 0, mc = 0, mini = 0;
  for (int l = l0; l < l1; l++) {
    ncap = std::max(ncap, lv[l].key_cap + 4);
    mc = std::max(mc, lv[l].ncells);
    mini = std::max(mini, lv[l].nini);
  }
  int sc = 1;
  while (sc < std::max(std::max(ncap, 16 * mini), 24)) sc <<= 1;  // sk doubles as the [NW][nini] bucket tables and 3 x NW scan sums
  p.node_cap = ncap;
  p.sort_cap = sc;
  p.scan_cap = (std::max(ncap, mc) + 3) & ~3;
  const size_t fixed = sizeof(ONode) * 2 * ncap + sizeof(int4) * ncap + sizeof(int) * 3 * p.scan_cap +
                       sizeof(unsigned long long) * sc + sizeof(int) * OCT_MISC_INTS;
  const size_t budget = (size_t)budget_kb * 1024;
  p.key_lds_cap = fixed < budget ? (int)((budget - fixed) / 8) & ~63 : 0;
  if (key_cap_override >= 0) p.key_lds_cap = std::min(p.key_lds_cap, key_cap_override);
  p.lds = fixed + sizeof(uint32_t) * 2 * (size_t)p.key_lds_cap;
  return p;
}

static void free_batch(orbfe_extractor* h) {
  if (h->hpyr_pending) {  // the host-pyramid prefetch still reads d_pyr
    hipEventSynchronize(h->ev_hpyr);
    h->hpyr_pending = false;
  }
  drop_graphs(h);
  hipFree(h->d_pyr);
  hipFree(h->d_blur);
  hipFree(h->d_cand);
  hipFree(h->d_cellcnt);
  hipFree(h->d_keys_a);
  hipFree(h->d_keys_b);
  hipFree(h->d_lvlkeys);
  hipFree(h->d_lvlcnt);
  h->d_pyr = nullptr;
  h->d_blur = nullptr;
  h->d_cand = nullptr;
  h->d_cellcnt = nullptr;
  h->d_keys_a = h->d_keys_b = nullptr;
  h->d_lvlkeys = nullptr;
  h->d_lvlcnt = nullptr;
  h->batch_cap = 0;
}

static int ensure_batch(orbfe_extractor* h, int n) {
  if (n <= h->batch_cap) return ORBFE_OK;
  free_batch(h);
  const int cap = std::max(n, 1);
  // (+256: k_fast's 16-byte ROI loads may run up to 15 bytes past the last row of the block)
  ORBFE_HIP_CHECK(hipMalloc(&h->d_pyr, (size_t)h->pyr_stride * cap + 256));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_blur, (size_t)h->pyr_stride * cap + 256));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_cand, (size_t)h->cand_stride * 4 * cap));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_cellcnt, sizeof(int32_t) * h->cells.size() * cap + 4));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_keys_a, (size_t)h->keyscr_stride * 4 * cap));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_keys_b, (size_t)h->keyscr_stride * 4 * cap));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_lvlkeys, (size_t)h->lvlkey_stride * 4 * cap));
  ORBFE_HIP_CHECK(hipMalloc(&h->d_lvlcnt, sizeof(int32_t) * h->nlevels * cap));
  h->batch_cap = cap;
  return ORBFE_OK;
}

static size_t octree_lds(const orbfe_extractor* h) {
  return h->oct_all.lds;
}
// constant 68-byte ROI rows when every cell ROI fits (xo <= 3 alignment bytes + rw <= 61) and the
// multiply-shift row split stays exact (dw^2 * dh < 2^20)
static int fast_rs(const orbfe_extractor* h) {
  return (h->roi_w_max <= 61 && h->roi_h_max <= 66) ? 68 : 0;
}
static size_t fast_lds(const orbfe_extractor* h) {
  return 4 * (size_t)fast_lds_layout(h->roi_w_max, h->roi_h_max, fast_rs(h)).total;
}

// How many levels, from level 0 up, get their FAST launch on the side stream as soon as the main
// stream has built them; the rest run in one launch after the resize chain. Measured on MI355X
// (C3 bench, stereo frames/s): 1 level 67.6k, 2 levels 68.7k, 3 levels 69.1-69.4k, 4 levels
// 69.0k, 5 66.6k, 8 60.3k -- the big levels' FAST fills the CUs the latency-bound resize chain
// leaves idle, the small ones only stretch the chain.
static int fast_side_split(const orbfe_extractor* h) {
  return std::min(h->fast_side_levels > 0 ? h->fast_side_levels : 3, h->nlevels);
}

// Images i0..i0+n-1 of the handle's per-image scratch (pyramid, candidates, octree keys) hold
// this launch's n images; d_imgs and the outputs are the caller's pointers for exactly these n.
static int launch_extract(orbfe_extractor* h, int n, const uint8_t* d_imgs, long long img_stride,
                          int pitch, orbfe_keypoint* d_kps, uint8_t* d_desc, int cap,
                          int32_t* d_counts, hipStream_t st, int i0 = 0) {
  // the handle's high-priority side stream (k_blur and the early FAST levels beside the main chain),
  // or the launch stream itself when the caller overlaps whole extractions instead
  // (orbfe_debug_set_inline_side)
  const hipStream_t side = (h->inline_side || (h->call_inline && n < 8)) ? st : (h->side_ext ? h->side_ext : h->side);
  ExtractArgs a;
  std::memset(&a, 0, sizeof(a));
  a.levels = h->d_levels;
  a.cells = h->d_cells;
  a.xtab = h->d_xtab;
  a.ytab = h->d_ytab;
  a.ywin = h->d_ywin;
  a.nlevels = h->nlevels;
  a.ncells = (int)h->cells.size();
  a.n_images = n;
  a.total_key_slots = h->total_key_slots;
  a.blur_strips = h->blur_tiles;
  a.img0 = d_imgs;
  a.img_stride = img_stride;
  a.img_pitch = pitch;
  a.pyr = h->d_pyr + (long long)i0 * h->pyr_stride;
  a.blur = h->d_blur + (long long)i0 * h->pyr_stride;
  a.pyr_stride = h->pyr_stride;
  a.cand = h->d_cand + (long long)i0 * h->cand_stride;
  a.cand_stride = h->cand_stride;
  a.cellcnt = h->d_cellcnt + (long long)i0 * h->cells.size();
  a.keys_a = h->d_keys_a + (long long)i0 * h->keyscr_stride;
  a.keys_b = h->d_keys_b + (long long)i0 * h->keyscr_stride;
  a.keyscr_stride = h->keyscr_stride;
  a.lvlkeys = h->d_lvlkeys + (long long)i0 * h->lvlkey_stride;
  a.lvlkey_stride = h->lvlkey_stride;
  a.lvlcnt = h->d_lvlcnt + (long long)i0 * h->nlevels;
  a.out_kps = d_kps;
  a.out_desc = d_desc;
  a.out_counts = d_counts;
  a.out_cap = cap;
  a.ini_th = h->ini_th;
  a.min_th = h->min_th;
  a.roi_w_max = h->roi_w_max;
  a.roi_h_max = h->roi_h_max;
  a.node_cap = h->node_cap;
  a.sort_cap = h->sort_cap;
  a.scan_cap = h->scan_cap;
  a.key_lds_cap = h->key_lds_cap;
  a.rgrp = h->d_rgrp;
  a.rgx0 = h->d_rgx0;
  for (int v = 0; v < 16; v++) a.umax[v] = h->umax[v];
  a.atan.p1 = 0.9997878412794807f * (float)(180 / M_PI);
  a.atan.p3 = -0.3258083974640975f * (float)(180 / M_PI);
  a.atan.p5 = 0.1555786518463281f * (float)(180 / M_PI);
  a.atan.p7 = -0.04432655554792128f * (float)(180 / M_PI);
  a.atan.eps = (float)DBL_EPSILON;
  a.factor_pi = (float)(M_PI / 180.f);

  auto launch_fast = [&](hipStream_t s, int c0, int c1, bool main_launch = false) -> int {
    if (c1 <= c0) return ORBFE_OK;
    // wavefronts (cells) per workgroup: 4 for the side-stream launches of levels 0-2, which run
    // beside the resize chain (smaller workgroups there take CUs from it: 1 per workgroup made
    // k_fast 176 -> 161 us alone but k_resize 146 -> 177 us); 1 for the levels-3..7 launch after
    // the chain (bench 77.4 / 77.6k vs 76.5 / 76.8k stereo frames/s, interleaved; 8 per workgroup
    // everywhere: 71.3k). profiles/scripts/r3_fast_wpb.sh
    const int wpb = main_launch ? h->fast_wpb_main : h->fast_wpb_side;
    dim3 grid((c1 - c0 + wpb - 1) / wpb, n);
    const size_t lds = fast_lds(h) / 4 * wpb;
    if (fast_rs(h) == 68)
      ORBFE_LAUNCH("k_fast", k_fast<68>, grid, dim3(64 * wpb), lds, s, a, c0, c1);
    else
      ORBFE_LAUNCH("k_fast", k_fast<0>, grid, dim3(64 * wpb), lds, s, a, c0, c1);
    return ORBFE_OK;
  };
  {
    const LevelDesc& d = h->levels[0];
    if (h->input_l0) {
      dim3 grid(((d.pitch * d.h) / 16 + 1023) / 1024, n);
      ORBFE_LAUNCH("k_copy_l0", k_copy_l0, grid, dim3(256), 0, st, a);
    } else {
      dim3 grid((d.h + 3) / 4, n);
      const size_t lds = 4 * sizeof(uint32_t) * (size_t)((d.pitch >> 2) + 4);
      ORBFE_LAUNCH("k_copy0", k_copy0, grid, dim3(256), lds, st, a);
    }
  }
  // the FAST cells of levels 0..k-1 run on the side stream, each level as soon as the main stream
  // has built it, beside the chain of small dependent resize launches that leaves most CUs idle;
  // levels k..L-1 follow the chain on the main stream
  // latency schedule (orbfe_debug_set_latency_schedule, calls of fewer than 8 images): FAST of
  // levels 0..k-1 and then their DistributeOctTree on the side stream, beside the main stream's
  // resize chain, FAST and octree of levels k..L-1 (both octree launches at the full LDS plan);
  // joined before k_describe. Level 0's octree block, the longest, starts right after its FAST
  // instead of after the whole pyramid's: one KITTI image 0.169-0.181 vs 0.189-0.201 ms per
  // orbfe_extract at k = 1 (k = 2 1-3 us slower in 3 of 4 A/B runs, k = 3 0.185-0.194; enqueueing
  // the side's work after the main chain's: no gain at k = 2, far slower at 1 and 3;
  // profiles/r5_c2_sched.txt)
  const bool lat = h->lat_sched > 0 && h->lat_sched < h->nlevels && n < 8;
  const int k_side = lat ? h->lat_sched : fast_side_split(h);
  if ((int)h->ev_lvl.size() < h->nlevels) {
    for (int l = (int)h->ev_lvl.size(); l < h->nlevels; l++) {
      hipEvent_t e = nullptr;
      ORBFE_HIP_CHECK(hipEventCreateWithFlags(&e, kForkJoinEvent));
      h->ev_lvl.push_back(e);
    }
  }
  auto side_fast = [&](int l) -> int {
    const hipEvent_t e = l == 0 ? h->ev_l0 : h->ev_lvl[l];
    ORBFE_HIP_CHECK(hipEventRecord(e, st));
    ORBFE_HIP_CHECK(hipStreamWaitEvent(side, e, 0));
    const int c1 = l + 1 < h->nlevels ? h->levels[l + 1].cell_begin : a.ncells;
    return launch_fast(side, h->levels[l].cell_begin, c1);
  };
  if (std::max(h->oct_all.lds, std::max(h->oct_hi.lds, h->oct_lo.lds)) > 160 * 1024)
    return orbfe_set_error(ORBFE_ERR_ARG, "image too large for the octree LDS plan");
  auto launch_octree = [&](hipStream_t s, int l0, int nl, const OctPlan& P) {
    if (nl <= 0) return;
    ExtractArgs ao = a;
    ao.node_cap = P.node_cap;
    ao.sort_cap = P.sort_cap;
    ao.scan_cap = P.scan_cap;
    ao.key_lds_cap = P.key_lds_cap;
    ao.oct_small = n >= 8 ? h->oct_small_batch : h->oct_small_small;
    dim3 grid(nl, n);
    // calls of fewer than 8 images leave the chip nearly idle: one 512-thread block per level (8
    // wavefronts share each pass's node splits and the refinement's child counts, partitions and
    // rank sort), against 256 threads for batches, where the blocks run beside other kernels. One
    // KITTI image: the octree's two launches 84.6 us summed at 512 vs 95.4 at 256 and 92.9 at 1024
    // threads (16 wavefronts pay more per barrier and spill 2 VGPRs); orbfe_extract p50 0.196 vs
    // 0.198 / 0.202 ms (profiles/r6_c2_octree.txt)
    const int nt = n >= 8 ? h->oct_threads_batch : (l0 == 0 && h->oct_threads_l0 > 0) ? h->oct_threads_l0 : h->oct_threads_small;
    if (nt == 1024)
      ORBFE_LAUNCH("k_octree", k_octree<1024>, grid, dim3(1024), P.lds, s, ao, l0);
    else if (nt == 512)
      ORBFE_LAUNCH("k_octree", k_octree<512>, grid, dim3(512), P.lds, s, ao, l0);
    else
      ORBFE_LAUNCH("k_octree", k_octree<256>, grid, dim3(256), P.lds, s, ao, l0);
  };
  side_fast(0);
  if (lat && k_side == 1) launch_octree(side, 0, 1, h->oct_all);
  const orbfe_extractor::PyrPlan& pp = n < 8 ? h->pyr_small : h->pyr_batch;
  if (pp.ntiles > 0) {
    // levels 1..L-1 in one launch (k_pyramid); the side's FAST levels 1..k-1 then in one launch
    #ifdef ORBFE_PYR_CLOCKS
    static const int pyr_dbg = getenv("ORBFE_PYR_CLOCKS") ? 1 : 0;  // phase clocks (a timing build)
#else
    constexpr int pyr_dbg = 0;
#endif
    ORBFE_LAUNCH("k_pyramid", k_pyramid, dim3(pp.ntiles, n), dim3(PYR_NT), pp.lds, st, a, pp.d_tiles, pp.half_dw, pyr_dbg);
    if (k_side > 1) {
      const hipEvent_t e = h->ev_lvl[1];
      ORBFE_HIP_CHECK(hipEventRecord(e, st));
      ORBFE_HIP_CHECK(hipStreamWaitEvent(side, e, 0));
      const int st_ = launch_fast(side, h->levels[1].cell_begin,
                                  k_side < h->nlevels ? h->levels[k_side].cell_begin : a.ncells);
      if (st_ != ORBFE_OK) return st_;
      if (lat) launch_octree(side, 0, k_side, h->oct_all);
    }
  }
  for (int l = 1; l < h->nlevels && pp.ntiles == 0; l++) {
    const LevelDesc& d = h->levels[l];
    if (d.rwin_ok) {
      const int G = (d.w + 3) / 4, items = G * ((d.h + 1) / 2);
      const uint32_t gm = G > 1 ? (uint32_t)((0x100000000ull + G - 1) / G) : 0u;  // exact: items * G < 2^32
      dim3 grid((items + 255) / 256, n);
      ORBFE_LAUNCH("k_resize_win", k_resize_win, grid, dim3(256), 0, st, a, l, G, gm);
    } else {
      dim3 grid((d.w + 255) / 256, (d.h + 4 * RESIZE_ROWS - 1) / (4 * RESIZE_ROWS), n), block(64, 4);
      ORBFE_LAUNCH("k_resize", k_resize, grid, block, 0, st, a, l);
    }
    if (l < k_side) {
      if (!h->fast_side_merge || lat) {
        side_fast(l);
      } else if (l == k_side - 1) {  // levels 1..k-1 in one side launch once level k-1 is built
        ORBFE_HIP_CHECK(hipEventRecord(h->ev_lvl[l], st));
        ORBFE_HIP_CHECK(hipStreamWaitEvent(side, h->ev_lvl[l], 0));
        const int c1 = l + 1 < h->nlevels ? h->levels[l + 1].cell_begin : a.ncells;
        const int r = launch_fast(side, h->levels[1].cell_begin, c1);
        if (r != ORBFE_OK) return r;
      }
    }
    if (lat && l == k_side - 1) launch_octree(side, 0, k_side, h->oct_all);
  }
  // main: FAST of the other levels, then the side's FAST levels joined. Fork: GaussianBlur needs
  // only the pyramid, so it runs on the side stream beside k_octree (a small, latency-bound grid
  // that leaves most CUs idle); joined before k_describe. (Measured on MI355X and not kept:
  // DistributeOctTree of the side's levels on the side stream right after their FAST, beside the
  // main stream's FAST -- bench 63.7k vs 67.0k stereo frames/s, it competes with that FAST; the
  // blur on the side stream as soon as the pyramid is complete -- 65.1k vs 69.3-70.0k.)
  // the pyramid is complete on st (under capture this record is only a graph-internal dependency:
  // launch_extract_graphed records the event again after the graph launch)
  ORBFE_HIP_CHECK(hipEventRecord(h->ev_pyr, st));
  const int blur_wpb = 4;  // 1 or 2 strips per workgroup: no difference (76.4-77.0k vs 77.2k)
  const dim3 blur_grid((h->blur_tiles + blur_wpb - 1) / blur_wpb, n);
  ORBFE_HIP_CHECK(hipEventRecord(h->ev_f0, side));
  // (latency schedule: the blur follows the side's octree as soon as the pyramid is complete)
  if (lat && h->blur_mode == 0) ORBFE_HIP_CHECK(hipEventRecord(h->ev_fork, st));
  if (k_side < h->nlevels) launch_fast(st, h->levels[k_side].cell_begin, a.ncells, true);
  if (!lat) ORBFE_HIP_CHECK(hipStreamWaitEvent(st, h->ev_f0, 0));
  if (h->blur_mode == 0) {  // the blur on the side stream beside DistributeOctTree
    if (!lat) ORBFE_HIP_CHECK(hipEventRecord(h->ev_fork, st));
    ORBFE_HIP_CHECK(hipStreamWaitEvent(side, h->ev_fork, 0));
    ORBFE_LAUNCH("k_blur", k_blur, blur_grid, dim3(64 * blur_wpb), 0, side, a);
    ORBFE_HIP_CHECK(hipEventRecord(h->ev_join, side));
  }
  {
    // two launches only for device-resident batches (the entry point of callers that overlap
    // extractions): they cut the LDS the short small-level blocks hold, which pays when other
    // kernels run beside the octree (the C3 bench: 85.4-85.5k vs 84.0-84.1k stereo frames/s,
    // interleaved, round 5); alone, one extraction's octree then runs as two dependent launches
    // (the launch span 116 vs 69 us), so single images and the synchronous host-buffer calls
    // keep one launch
    const int ks = (h->device_call && n >= 8) ? std::min(std::max(h->octree_split, 0), h->nlevels) : 0;
    if (lat) {
      launch_octree(st, k_side, h->nlevels - k_side, h->oct_all);
    } else if (ks > 0 && ks < h->nlevels) {
      launch_octree(st, 0, ks, h->oct_hi);
      launch_octree(st, ks, h->nlevels - ks, h->oct_lo);
    } else {
      launch_octree(st, 0, h->nlevels, h->oct_all);
    }
  }
  if (h->blur_mode == 1)  // the blur after DistributeOctTree on the launch stream
    ORBFE_LAUNCH("k_blur", k_blur, blur_grid, dim3(64 * blur_wpb), 0, st, a);
  if (h->blur_mode == 0) ORBFE_HIP_CHECK(hipStreamWaitEvent(st, h->ev_join, 0));
  if (lat && h->blur_mode != 0) ORBFE_HIP_CHECK(hipStreamWaitEvent(st, h->ev_f0, 0));  // the side's octree
  {
    constexpr int per_block = 4 * DESC_WPB;  // keypoints per workgroup
    dim3 grid((h->total_key_slots + per_block - 1) / per_block, n);
    ORBFE_LAUNCH("k_describe", k_describe, grid, dim3(DESC_THREADS), 0, st, a);
  }
  ORBFE_HIP_CHECK(hipGetLastError());
  h->last_img0 = d_imgs - (long long)i0 * img_stride;
  h->last_img_stride = img_stride;
  h->last_img_pitch = pitch;
  h->last_n = i0 + n;
  h->last_stream = st;
  return ORBFE_OK;
}

// launch_extract through a hipGraph: the enqueue sequence (about 20 kernel launches and the side
// stream's fork / join events) is captured from the launch stream the first time a set of
// arguments is seen, instantiated, and replayed with one hipGraphLaunch afterwards. The key holds
// every input the sequence depends on: the caller's pointers, strides and stream, the handle's
// scratch (reallocated buffers change it), streams and placement switches. Launches stay direct
// while the kernel timer is on (its per-dispatch events cannot be captured), while the stream is
// already being captured by the caller, or after a capture failed on this handle.
constexpr size_t kMaxGraphs = 8;
static int launch_extract_graphed(orbfe_extractor* h, int n, const uint8_t* d_imgs, long long img_stride,
                                  int pitch, orbfe_keypoint* d_kps, uint8_t* d_desc, int cap,
                                  int32_t* d_counts, hipStream_t st, int i0 = 0) {
  // the per-level fork events exist before any capture
  while ((int)h->ev_lvl.size() < h->nlevels) {
    hipEvent_t e = nullptr;
    ORBFE_HIP_CHECK(hipEventCreateWithFlags(&e, kForkJoinEvent));
    h->ev_lvl.push_back(e);
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  // direct launches when the side stream is a caller's shared one (orbfe_set_side_stream): a
  // capture pulls the side stream in through the fork / join events, and the other handles'
  // launches onto it from their threads would collide with the capture
  if (!h->use_graphs || !st || h->side_ext || orbfe_kt::g_on.load(std::memory_order_relaxed) ||
      hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return launch_extract(h, n, d_imgs, img_stride, pitch, d_kps, d_desc, cap, d_counts, st, i0);
  const hipStream_t side = h->inline_side ? st : (h->side_ext ? h->side_ext : h->side);
  const std::vector<uintptr_t> key = {
      (uintptr_t)n, (uintptr_t)d_imgs, (uintptr_t)img_stride, (uintptr_t)pitch, (uintptr_t)d_kps,
      (uintptr_t)d_desc, (uintptr_t)cap, (uintptr_t)d_counts, (uintptr_t)st, (uintptr_t)i0, (uintptr_t)side,
      (uintptr_t)h->rows, (uintptr_t)h->cols, (uintptr_t)h->geom_mode, (uintptr_t)h->d_levels,
      (uintptr_t)h->d_pyr, (uintptr_t)h->d_blur, (uintptr_t)h->d_cand, (uintptr_t)h->d_cellcnt,
      (uintptr_t)h->d_keys_a, (uintptr_t)h->d_keys_b, (uintptr_t)h->d_lvlkeys, (uintptr_t)h->d_lvlcnt,
      (uintptr_t)h->key_lds_cap, (uintptr_t)h->octree_split, (uintptr_t)(h->oct_hi_kb * 1024 + h->oct_lo_kb), (uintptr_t)h->device_call, (uintptr_t)(h->fast_wpb_side * 16 + h->fast_wpb_main), (uintptr_t)h->fast_side_levels, (uintptr_t)h->fast_side_merge, (uintptr_t)h->input_l0, (uintptr_t)h->inline_side, (uintptr_t)(h->oct_threads_small * 4096 + h->oct_threads_batch), (uintptr_t)h->pyr_small.d_tiles, (uintptr_t)h->pyr_batch.d_tiles,
      (uintptr_t)h->blur_mode};
  h->graph_clock++;
  hipGraphExec_t exec = nullptr;
  for (auto& e : h->graphs)
    if (e.key == key) {
      exec = e.exec;
      e.used = h->graph_clock;
      h->graph_hits++;
      break;
    }
  if (!exec) {
    hipGraph_t g = nullptr;
    ORBFE_HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    const int r = launch_extract(h, n, d_imgs, img_stride, pitch, d_kps, d_desc, cap, d_counts, st, i0);
    const hipError_t ee = hipStreamEndCapture(st, &g);
    hipError_t ie = hipErrorUnknown;
    if (r == ORBFE_OK && ee == hipSuccess && g) ie = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    if (g) hipGraphDestroy(g);
    if (r != ORBFE_OK) return r;
    if (ee != hipSuccess || ie != hipSuccess) {  // this handle launches directly from now on
      (void)hipGetLastError();
      h->use_graphs = 0;
      return launch_extract(h, n, d_imgs, img_stride, pitch, d_kps, d_desc, cap, d_counts, st, i0);
    }
    if (h->graphs.size() >= kMaxGraphs) {
      auto lru = std::min_element(h->graphs.begin(), h->graphs.end(),
                                  [](const orbfe_extractor::GraphEntry& a, const orbfe_extractor::GraphEntry& b) {
                                    return a.used < b.used;
                                  });
      hipGraphExecDestroy(lru->exec);
      h->graphs.erase(lru);
    }
    h->graphs.push_back({key, exec, h->graph_clock});
    h->graph_captures++;
  }
  ORBFE_HIP_CHECK(hipGraphLaunch(exec, st));
  // for the callers that wait on the pyramid event (the host pyramid prefetch, other streams'
  // consumers of orbfe_extractor_pyramid_event): recorded after the whole replayed extraction, a
  // later point than the direct launches' record after the resize chain. (Capturing the record as
  // an external event node, hipEventRecordWithFlags(..., hipEventRecordExternal), failed with
  // "invalid argument" in the host-fed pipeline on ROCm 7.2.)
  ORBFE_HIP_CHECK(hipEventRecord(h->ev_pyr, st));
  h->last_img0 = d_imgs - (long long)i0 * img_stride;
  h->last_img_stride = img_stride;
  h->last_img_pitch = pitch;
  h->last_n = i0 + n;
  h->last_stream = st;
  return ORBFE_OK;
}

// A new call rewrites d_pyr: its launches on `s` wait for the previous call's host-pyramid
// prefetch copies (h->d2h), which only orbfe_get_level otherwise waits for.
static int wait_host_pyramid(orbfe_extractor* h, hipStream_t s) {
  if (h->hpyr_pending) ORBFE_HIP_CHECK(hipStreamWaitEvent(s, h->ev_hpyr, 0));
  return ORBFE_OK;
}

static void drop_graphs(orbfe_extractor* h) {
  for (auto& e : h->graphs) hipGraphExecDestroy(e.exec);
  h->graphs.clear();
}

// The host block of orbfe_get_level, sized for n images of the current geometry. Called once per
// extract call before any image of that call is copied into it, so a reallocation never moves a
// level the caller still holds from the same call.
static int ensure_host_pyramid(orbfe_extractor* h, int n) {
  const size_t need = (size_t)h->pyr_stride * n;
  if (need > h->h_pyr_bytes) {
    if (h->hpyr_pending) {
      ORBFE_HIP_CHECK(hipEventSynchronize(h->ev_hpyr));
      h->hpyr_pending = false;
    }
    if (h->h_pyr) hipHostFree(h->h_pyr);
    h->h_pyr = nullptr;
    h->h_pyr_bytes = 0;
    ORBFE_HIP_CHECK(hipHostMalloc((void**)&h->h_pyr, need, hipHostMallocDefault));
    h->h_pyr_bytes = need;
  }
  if ((int)h->h_pyr_gen.size() < n) h->h_pyr_gen.resize(n, 0);
  if (!h->ev_hpyr) ORBFE_HIP_CHECK(hipEventCreateWithFlags(&h->ev_hpyr, hipEventDisableTiming));
  return ORBFE_OK;
}

// ---------------------------------------------------------------------------------------------
// C ABI
// The side stream gets the highest priority: the runtime serves each priority from its own
// hardware queues, so k_blur cannot land behind the caller's stream on a shared queue.
// ORBFE_DEDICATED_QUEUES=1: a handle's own streams (the launch stream and the side stream of its
// host-buffer calls, the copy streams of large host batches) each get a hardware queue of their own
// -- a stream created with a CU mask (here: every CU) is not placed on the runtime's shared pool
// (GPU_MAX_HW_QUEUES, 4 by default). On the pool, with 4+ idle extractor handles alive, one image
// through orbfe_extract took 0.275-0.283 vs 0.130-0.135 ms p50 (idle torch streams of either
// priority did not do it); with dedicated queues 0.130 at any handle count
// (profiles/r6_c2_queues.txt). Not the default: in the bench process, whose legs create many
// handles, the extra queues slowed the host-fed C3 leg 48.6k -> 22.9k stereo frames/s, the tracking
// leg 978 -> 511 frames/s and C5 2,736 -> 429 (hardware queue oversubscription).
static hipError_t create_masked_stream(hipStream_t* s) {
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return hipErrorUnknown;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
  return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}
static bool cu_mask_streams() {
  static const bool on = std::getenv("ORBFE_DEDICATED_QUEUES") != nullptr;
  return on;
}
static hipError_t create_side_stream(hipStream_t* s) {
  if (cu_mask_streams()) return create_masked_stream(s);
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
}
static hipError_t create_main_stream(hipStream_t* s) {
  if (cu_mask_streams()) return create_masked_stream(s);
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}


extern "C" int orbfe_extractor_create(int nfeatures, float scale_factor, int nlevels,
                                      int ini_th_fast, int min_th_fast, int device,
                                      orbfe_extractor** out) {
  if (!out || nfeatures <= 0 || nlevels <= 0 || nlevels > 32 || !(scale_factor > 1.0f))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extractor_create: bad argument");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_extractor_create: no HIP device");
  if (device < 0 || device >= ndev) return orbfe_set_error(ORBFE_ERR_ARG, "bad device index");
  orbfe_extractor* h = new orbfe_extractor();
  h->device = device;
  {
    const char* e = std::getenv("ORBFE_SCHED_AUTOTUNE");
    h->autotune = (e && e[0] == '0') ? 0 : 1;
    const char* o = std::getenv("ORBFE_OCT_THREADS_SMALL");  // (A/B runs of whole processes)
    if (o && (std::atoi(o) == 256 || std::atoi(o) == 512 || std::atoi(o) == 1024)) h->oct_threads_small = std::atoi(o);
    const char* q = std::getenv("ORBFE_OCT_SERIAL_SMALL");  // (A/B runs of whole processes)
    if (q && std::atoi(q) >= 1 && std::atoi(q) <= OCT_SMALL_MAX) h->oct_small_small = std::atoi(q);
  }
  h->nfeatures = nfeatures;
  h->nlevels = nlevels;
  h->ini_th = ini_th_fast;
  h->min_th = min_th_fast;
  // ORBextractor::ORBextractor (ORBextractor.cc:413-473); scaleFactor is a double member
  h->scale_factor = (double)scale_factor;
  h->scale.assign(nlevels, 1.0f);
  h->sigma2.assign(nlevels, 1.0f);
  for (int i = 1; i < nlevels; i++) {
    h->scale[i] = (float)((double)h->scale[i - 1] * h->scale_factor);
    h->sigma2[i] = h->scale[i] * h->scale[i];
  }
  h->inv_scale.resize(nlevels);
  h->inv_sigma2.resize(nlevels);
  for (int i = 0; i < nlevels; i++) {
    h->inv_scale[i] = 1.0f / h->scale[i];
    h->inv_sigma2[i] = 1.0f / h->sigma2[i];
  }
  h->nfeat.resize(nlevels);
  const float factor = (float)(1.0 / h->scale_factor);
  float nd = (float)nfeatures * (1.0f - factor) / (1.0f - (float)std::pow((double)factor, (double)nlevels));
  int sum = 0;
  for (int l = 0; l < nlevels - 1; l++) {
    h->nfeat[l] = h_round(nd);
    sum += h->nfeat[l];
    nd *= factor;
  }
  h->nfeat[nlevels - 1] = std::max(nfeatures - sum, 0);
  int v, v0, vmax = h_floor(15 * std::sqrt(2.f) / 2 + 1);
  const float vminf = 15 * std::sqrt(2.f) / 2;
  int vmin = (int)vminf;
  vmin += (vmin < vminf);
  for (v = 0; v <= vmax; ++v) h->umax[v] = (int)std::lrint(std::sqrt(225.0 - v * v));
  for (v = 15, v0 = 0; v >= vmin; --v) {
    while (h->umax[v0] == h->umax[v0 + 1]) ++v0;
    h->umax[v] = v0;
    ++v0;
  }
  if (hipSetDevice(device) != hipSuccess ||
      create_main_stream(&h->stream) != hipSuccess ||
      create_side_stream(&h->side) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_fork, kForkJoinEvent) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_join, kForkJoinEvent) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_l0, kForkJoinEvent) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_f0, kForkJoinEvent) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_pyr, hipEventDisableTiming) != hipSuccess) {
    delete h;
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_extractor_create: stream creation failed");
  }
  static std::once_flag once;
  static hipError_t pat_err = hipSuccess;
  std::call_once(once, [h] {
    pat_err = hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), kOrbPattern31, 1024);
    float patf[1024];
    for (int i = 0; i < 1024; i++) patf[i] = (float)kOrbPattern31[i];
    if (pat_err == hipSuccess) pat_err = hipMemcpyToSymbol(HIP_SYMBOL(c_patf), patf, sizeof(patf));
    // IC_Angle's circle |u| <= umax[|v|], v = -15..15: 749 pixels (the kernel builds each window
    // dword's byte mask from these 4-bit fields)
    uint32_t um4[2] = {0u, 0u};
    int npx = 0;
    for (int v = -15; v <= 15; v++) npx += 2 * h->umax[std::abs(v)] + 1;
    for (int v = 0; v < 16; v++) um4[v >> 3] |= (uint32_t)h->umax[v] << (4 * (v & 7));
    if (pat_err == hipSuccess && npx == 749) pat_err = hipMemcpyToSymbol(HIP_SYMBOL(c_umax4), um4, sizeof(um4));
    else if (pat_err == hipSuccess) pat_err = hipErrorInvalidValue;
  });
  if (pat_err != hipSuccess) {
    delete h;
    return orbfe_set_hip_error(pat_err, "upload pattern");
  }
  *out = h;
  return ORBFE_OK;
}

extern "C" int orbfe_extractor_destroy(orbfe_extractor* h) {
  if (!h) return ORBFE_OK;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->h2d) hipStreamSynchronize(h->h2d);
  if (h->d2h) hipStreamSynchronize(h->d2h);  // (the host-pyramid prefetch reads d_pyr)
  orbfe_internal_stereo_free(h->stereo);
  drop_graphs(h);
  free_batch(h);
  hipFree(h->d_levels);
  hipFree(h->d_cells);
  hipFree(h->d_xtab);
  hipFree(h->d_ytab);
  hipFree(h->d_ywin);
  hipFree(h->d_rgrp);
  hipFree(h->d_rgx0);
  hipFree(h->pyr_small.d_tiles);
  hipFree(h->pyr_batch.d_tiles);
  hipFree(h->d_in);
  hipFree(h->d_out);
  if (h->h_in) hipHostFree(h->h_in);
  if (h->h_out) hipHostFree(h->h_out);
  if (h->h_pyr) hipHostFree(h->h_pyr);
  if (h->ev_hpyr) hipEventDestroy(h->ev_hpyr);
  delete h->pool;
  for (auto e : h->ev_in) hipEventDestroy(e);
  for (auto e : h->ev_ext) hipEventDestroy(e);
  for (auto e : h->ev_out) hipEventDestroy(e);
  if (h->h2d) hipStreamDestroy(h->h2d);
  if (h->d2h) hipStreamDestroy(h->d2h);
  if (h->stream) hipStreamDestroy(h->stream);
  if (h->side) hipStreamDestroy(h->side);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  if (h->ev_l0) hipEventDestroy(h->ev_l0);
  if (h->ev_f0) hipEventDestroy(h->ev_f0);
  if (h->ev_pyr) hipEventDestroy(h->ev_pyr);
  for (hipEvent_t e : h->ev_lvl) hipEventDestroy(e);
  delete h;
  return ORBFE_OK;
}

extern "C" int orbfe_extractor_set_resize_mode(orbfe_extractor* h, int mode) {
  if (!h || (mode != ORBFE_RESIZE_SIMD128 && mode != ORBFE_RESIZE_SCALAR)) return ORBFE_ERR_ARG;
  h->resize_mode = mode;
  return ORBFE_OK;
}

extern "C" int orbfe_get_scale_tables(const orbfe_extractor* h, float* scale, float* inv_scale,
                                      float* sigma2, float* inv_sigma2, int32_t* fpl) {
  if (!h) return ORBFE_ERR_ARG;
  for (int l = 0; l < h->nlevels; l++) {
    if (scale) scale[l] = h->scale[l];
    if (inv_scale) inv_scale[l] = h->inv_scale[l];
    if (sigma2) sigma2[l] = h->sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = h->inv_sigma2[l];
    if (fpl) fpl[l] = h->nfeat[l];
  }
  return ORBFE_OK;
}

extern "C" int orbfe_max_keypoints(orbfe_extractor* h, int rows, int cols) {
  if (!h) return ORBFE_ERR_ARG;
  hipSetDevice(h->device);
  const int st = compute_geometry(h, rows, cols);
  if (st != ORBFE_OK) return st;
  return h->total_key_slots;
}

extern "C" void* orbfe_extractor_stream(orbfe_extractor* h) { return h ? (void*)h->stream : nullptr; }
extern "C" void* orbfe_extractor_pyramid_event(orbfe_extractor* h) { return h ? (void*)h->ev_pyr : nullptr; }
extern "C" int orbfe_stream_create(int device, int high_priority, void** out) {
  if (!out) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_stream_create: out is NULL");
  *out = nullptr;
  hipStream_t s = nullptr;
  ORBFE_HIP_CHECK(hipSetDevice(device));
  if (high_priority) {  // (a pooled stream at the highest priority, as requested)
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    ORBFE_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
  } else {
    ORBFE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  *out = (void*)s;
  return ORBFE_OK;
}

extern "C" int orbfe_stream_create_masked(int device, const uint32_t* cu_mask, int n_words, void** out) {
  if (!out || !cu_mask || n_words <= 0) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_stream_create_masked: bad argument");
  *out = nullptr;
  hipStream_t s = nullptr;
  ORBFE_HIP_CHECK(hipSetDevice(device));
  ORBFE_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, cu_mask));
  *out = (void*)s;
  return ORBFE_OK;
}

extern "C" int orbfe_stream_destroy(void* stream) {
  if (!stream) return ORBFE_OK;
  ORBFE_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  ORBFE_HIP_CHECK(hipStreamDestroy((hipStream_t)stream));
  return ORBFE_OK;
}

extern "C" int orbfe_event_create(int device, void** out) {
  if (!out) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_event_create: out is NULL");
  *out = nullptr;
  hipEvent_t e = nullptr;
  ORBFE_HIP_CHECK(hipSetDevice(device));
  ORBFE_HIP_CHECK(hipEventCreateWithFlags(&e, kForkJoinEvent));
  *out = (void*)e;
  return ORBFE_OK;
}

extern "C" int orbfe_event_record(void* event, void* stream) {
  if (!event) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_event_record: null event");
  ORBFE_HIP_CHECK(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
  return ORBFE_OK;
}

extern "C" int orbfe_event_query(void* event) {
  if (!event) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_event_query: null event");
  const hipError_t e = hipEventQuery((hipEvent_t)event);
  if (e == hipErrorNotReady) {
    // a runtime that records NotReady as the thread's last error would fail the next
    // hipGetLastError check (a matcher's pending_err, ORBFE_HIP_CHECK) on this thread; an
    // earlier, real error stays recorded
    if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
    return 1;
  }
  ORBFE_HIP_CHECK(e);
  return 0;
}

extern "C" int orbfe_event_destroy(void* event) {
  if (event) ORBFE_HIP_CHECK(hipEventDestroy((hipEvent_t)event));
  return ORBFE_OK;
}

extern "C" int orbfe_stream_wait_event(void* stream, void* event) {
  if (!event) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_stream_wait_event: null event");
  ORBFE_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return ORBFE_OK;
}

extern "C" int orbfe_extract_batch_device(orbfe_extractor* h, int n, const uint8_t* d_imgs,
                                          size_t image_stride, int rows, int cols, size_t pitch,
                                          orbfe_keypoint* d_kps, uint8_t* d_desc, int cap,
                                          int32_t* d_counts, void* stream) {
  if (!h || n < 0 || !d_imgs || !d_kps || !d_desc || !d_counts || rows <= 0 || cols <= 0 ||
      pitch < (size_t)cols)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extract_batch_device: bad argument");
  if (n == 0) return ORBFE_OK;
  hipSetDevice(h->device);
  int st = compute_geometry(h, rows, cols);
  if (st != ORBFE_OK) return st;
  if (cap < h->total_key_slots) return orbfe_set_error(ORBFE_ERR_CAPACITY, "cap < orbfe_max_keypoints");
  st = ensure_batch(h, n);
  if (st != ORBFE_OK) return st;
  hipStream_t s = stream ? (hipStream_t)stream : h->stream;
  h->gen++;  // the host pyramid block of the previous call is stale from here on
  st = wait_host_pyramid(h, s);
  if (st != ORBFE_OK) return st;
  h->device_call = true;
  h->call_inline = n < 8 && h->autotune && h->tune[n].decided == 1;
  st = launch_extract_graphed(h, n, d_imgs, (long long)image_stride, (int)pitch, d_kps, d_desc, cap,
                              d_counts, s);
  h->device_call = false;
  return st;
}

static int ensure_host_io(orbfe_extractor* h, int n, int rows, int cols) {
  const size_t need_in = (size_t)n * rows * cols;
  // (the zero-copy staging of a small call holds each image in the level-0 layout)
  const size_t need_h_in = std::max(need_in, (size_t)n * h->levels[0].pitch * h->levels[0].h);
  if (need_in > h->in_bytes) {
    hipFree(h->d_in);
    h->d_in = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&h->d_in, need_in));
    h->in_bytes = need_in;
  }
  const size_t need_out = (size_t)n * h->total_key_slots;
  if (need_out > h->out_cap_alloc || n > h->out_n_alloc) {
    // (64-slot multiples keep the descriptor and count regions 256-byte aligned)
    const size_t cap = (std::max(need_out, h->out_cap_alloc) + 63) & ~(size_t)63;
    const int nn = std::max(n, h->out_n_alloc);
    const size_t bytes = cap * (sizeof(orbfe_keypoint) + 32) + sizeof(int32_t) * (size_t)nn;
    hipFree(h->d_out);
    h->d_out = nullptr;
    h->d_kps = nullptr;
    h->d_desc = nullptr;
    h->d_counts = nullptr;
    h->out_cap_alloc = 0;
    h->out_n_alloc = 0;
    if (h->h_out) hipHostFree(h->h_out);
    h->h_out = nullptr;
    h->h_out_dev = nullptr;
    h->h_out_bytes = 0;
    ORBFE_HIP_CHECK(hipMalloc(&h->d_out, bytes));
    ORBFE_HIP_CHECK(hipHostMalloc((void**)&h->h_out, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    ORBFE_HIP_CHECK(hipHostGetDevicePointer((void**)&h->h_out_dev, h->h_out, 0));
    h->d_kps = reinterpret_cast<orbfe_keypoint*>(h->d_out);
    h->d_desc = h->d_out + cap * sizeof(orbfe_keypoint);
    h->d_counts = reinterpret_cast<int32_t*>(h->d_desc + cap * 32);
    h->out_cap_alloc = cap;
    h->out_n_alloc = nn;
    h->out_bytes = h->h_out_bytes = bytes;
  }
  if (need_h_in > h->h_in_bytes) {
    if (h->h_in) hipHostFree(h->h_in);
    h->h_in = nullptr;
    h->h_in_dev = nullptr;
    // coherent (fine-grained): k_copy0's reads of it over PCIe are never served from a GPU cache
    ORBFE_HIP_CHECK(hipHostMalloc((void**)&h->h_in, need_h_in, hipHostMallocMapped | hipHostMallocCoherent));
    h->h_in_bytes = need_h_in;
    ORBFE_HIP_CHECK(hipHostGetDevicePointer((void**)&h->h_in_dev, h->h_in, 0));
  }
  return ORBFE_OK;
}

// ---- registered host buffers (orbfe_host_register): copied from / to directly, no staging
namespace {
std::mutex g_reg_mu;
std::vector<std::pair<uintptr_t, size_t>> g_reg;  // registered [begin, begin + bytes)

bool host_registered(const void* p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (const auto& r : g_reg)
    if (a >= r.first && a + bytes <= r.first + r.second) return true;
  return false;
}
}  // namespace

extern "C" int orbfe_host_register(const void* p, size_t bytes) {
  if (!p || bytes == 0) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_host_register: bad argument");
  if (host_registered(p, bytes)) return ORBFE_OK;
  ORBFE_HIP_CHECK(hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault));
  std::lock_guard<std::mutex> g(g_reg_mu);
  g_reg.emplace_back((uintptr_t)p, bytes);
  return ORBFE_OK;
}

extern "C" int orbfe_host_unregister(const void* p) {
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = std::find_if(g_reg.begin(), g_reg.end(), [&](const std::pair<uintptr_t, size_t>& r) {
      return r.first == (uintptr_t)p;
    });
    if (it == g_reg.end()) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_host_unregister: not registered");
    g_reg.erase(it);
  }
  ORBFE_HIP_CHECK(hipHostUnregister(const_cast<void*>(p)));
  return ORBFE_OK;
}

// Host-buffer batch (what the reference's ORBextractor::operator() costs a caller). The images go
// through pinned staging in chunks: chunk c's H2D copy (copy stream) overlaps chunk c+1's staging
// (row bands spread over the handle's host worker pool). One extraction of all images follows
// (one launch sequence fills the GPU far better than several small ones), then the results come
// back in pieces on a second copy stream while the host unpacks the previous piece's used slots
// into the caller's buffers. D2H moves every slot of a piece's images (the counts are not known
// on the host before).
static int ensure_pipeline(orbfe_extractor* h, int nchunks) {
  if (!h->pool) {
    const unsigned hc = std::thread::hardware_concurrency();
    h->pool = new HostPool((int)std::min(7u, hc > 1 ? hc - 1 : 0u));
  }
  if (!h->h2d) ORBFE_HIP_CHECK(create_main_stream(&h->h2d));  // (queues of their own: see create_masked_stream)
  if (!h->d2h) ORBFE_HIP_CHECK(create_main_stream(&h->d2h));
  while ((int)h->ev_in.size() < nchunks) {
    hipEvent_t a = nullptr, b = nullptr, c = nullptr;
    ORBFE_HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    ORBFE_HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    ORBFE_HIP_CHECK(hipEventCreateWithFlags(&c, hipEventDisableTiming));
    h->ev_in.push_back(a);
    h->ev_ext.push_back(b);
    h->ev_out.push_back(c);
  }
  return ORBFE_OK;
}

extern "C" int orbfe_extract_batch(orbfe_extractor* h, int n, const uint8_t* const* imgs,
                                   int rows, int cols, size_t step, orbfe_keypoint* kps,
                                   uint8_t* desc, int cap, int32_t* counts) {
  return orbfe_internal_extract_batch(h, n, imgs, rows, cols, step, kps, desc, cap, counts, {});
}

int orbfe_internal_extract_batch(orbfe_extractor* h, int n, const uint8_t* const* imgs, int rows, int cols,
                                 size_t step, orbfe_keypoint* kps, uint8_t* desc, int cap, int32_t* counts,
                                 const std::function<int()>& after_launch, orbfe_keypoint* const* kps_img,
                                 uint8_t* const* desc_img) {
  const bool per_image = kps_img && desc_img;
  if (per_image && n >= 8) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_internal_extract_batch: per-image outputs on a large batch");
  if (!h || n < 0 || !imgs || !counts) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extract_batch: bad argument");
  if (after_launch && n >= 8) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_internal_extract_batch: hook on a large batch");
  if (n == 0) return ORBFE_OK;
  if (rows == 0 || cols == 0) {  // empty image: operator() returns without output (:1044-1045)
    for (int i = 0; i < n; i++) counts[i] = 0;
    return ORBFE_OK;
  }
  if (rows < 0 || cols < 0 || step < (size_t)cols) return orbfe_set_error(ORBFE_ERR_ARG, "bad image shape");
  for (int i = 0; i < n; i++)
    if (!imgs[i]) return orbfe_set_error(ORBFE_ERR_ARG, "null image");
  hipSetDevice(h->device);
  int st = compute_geometry(h, rows, cols);
  if (st != ORBFE_OK) return st;
  st = ensure_batch(h, n);
  if (st != ORBFE_OK) return st;
  st = ensure_host_io(h, n, rows, cols);
  if (st != ORBFE_OK) return st;
  // H2D chunks of ~8 images; extraction in ngroups launch sequences (each starts when its images
  // have arrived, so the first overlaps the rest of the H2D); D2H in 2 pieces per group
  // One group: 2 groups of 32 measured slower on MI355X (1.98 vs 1.60 ms p50 for 64 KITTI
  // images; a 32-image extraction costs far more than half of a 64-image one), and so did
  // splitting the H2D chunks over both copy streams (1.71 ms).
  static const int env_groups = std::getenv("ORBFE_HOST_GROUPS") ? std::atoi(std::getenv("ORBFE_HOST_GROUPS")) : 0;
  // registered caller memory (orbfe_host_register): images DMA'd straight from the caller's rows
  // (step == cols), results DMA'd straight into the caller's buffers (cap == slots per image)
  bool direct_in = step == (size_t)cols;
  for (int i = 0; i < n && direct_in; i++) direct_in = host_registered(imgs[i], (size_t)rows * cols);
  const int K0 = h->total_key_slots;
  const bool direct_out = !per_image && cap == K0 && kps && desc &&
                          host_registered(kps, (size_t)n * cap * sizeof(orbfe_keypoint)) &&
                          host_registered(desc, (size_t)n * cap * 32);
  const int ngroups = env_groups > 0 ? std::min(env_groups, std::max(1, n / 8)) : 1;
  const int cpg = std::max(1, std::min(4, n / (8 * ngroups)));  // H2D chunks per group
  // small batches (a single image: orbfe_extract) stay on the handle's stream, in one piece:
  // the cross-stream event hops cost more latency than the overlap saves
  const bool small = n < 8;
  // (one KITTI image: orbfe_extract p50 0.152 with the input read over PCIe by k_copy0, 0.159 after
  // an H2D copy; profiles/r6_c2_zero_copy.txt)
  const bool zc_in = small && !direct_in && h->zc_in && h->h_in_dev;
  // zc_in == 2: the staging holds each image in the level-0 layout (k_copy_l0); 1: plain rows read by
  // k_copy0 (one KITTI image 0.141-0.144 vs 0.144-0.146 ms in the layout: the host's padding costs
  // what the straight copy saves; profiles/r6_c2_zero_copy.txt)
  const bool zc_l0 = zc_in && h->zc_in == 2;
  const size_t l0_bytes = zc_l0 ? (size_t)h->levels[0].pitch * h->levels[0].h : (size_t)rows * cols;  // staging image stride
  const int nchunks = ngroups * cpg, npieces = small ? 1 : 2 * ngroups;
  st = ensure_pipeline(h, std::max(nchunks, npieces));
  if (st != ORBFE_OK) return st;
  h->gen++;
  st = wait_host_pyramid(h, h->stream);
  if (st != ORBFE_OK) return st;
  if (h->host_pyramid) {
    st = ensure_host_pyramid(h, n);
    if (st != ORBFE_OK) return st;
  }
  const hipStream_t s_in = small ? h->stream : h->h2d, s_out = small ? h->stream : h->d2h;
  // the schedule autotune (orbfe_extractor::SchedTune): 4 warm-up calls (both arms), then
  // alternate two streams / one stream until each has 6 timings; one stream is kept if its mean
  // (the largest sample of each arm dropped) is below 0.9x. On a shared queue the two-stream
  // calls swing between ~180, ~290 and ~400 us (profiles/r6_c2_queues.txt), so the mean, not the
  // median, carries the penalty; on distinct queues both arms are steady (~137 vs ~185 us)
  orbfe_extractor::SchedTune* tune = nullptr;
  int tune_arm = -1;
  const auto t_call = std::chrono::steady_clock::now();
  h->call_inline = false;
  if (small && h->autotune && !h->inline_side && !h->side_ext && !h->use_graphs && h->lat_sched > 0) {
    tune = &h->tune[n];
    if (tune->decided >= 0) {
      h->call_inline = tune->decided == 1;
    } else {
      const int k = tune->calls++;
      if (k >= 4) tune_arm = k % 2;  // 0: two streams, 1: the launch stream
      h->call_inline = (k % 2) == 1;
    }
  }
  const int K = h->total_key_slots;
  const size_t img_bytes = (size_t)rows * cols;
  const int band = 64;  // staging rows per task
  const int bands = (rows + band - 1) / band;
  // (h_out mirrors the device block d_out: the same offsets)
  orbfe_keypoint* hk = reinterpret_cast<orbfe_keypoint*>(h->h_out);
  uint8_t* hd = h->h_out + (h->d_desc - h->d_out);
  int32_t* hc = reinterpret_cast<int32_t*>(h->h_out + (reinterpret_cast<uint8_t*>(h->d_counts) - h->d_out));
  // a small call through the staging mirror takes its results down in one copy of the block's
  // prefix when the block is not much larger than the call (one copy engine transfer instead of
  // three, the counts' through a blit kernel among them: one image 0.17-0.18 vs 0.18-0.20 ms)
  const bool one_copy = small && !direct_out && h->out_cap_alloc <= 2 * (size_t)n * K + 64;
  // (zero copy out: the kernels' result stores cross PCIe as they happen; with zero copy in 0.134
  // vs 0.152 ms p50, profiles/r6_c2_zero_copy.txt)
  const bool zc_out = one_copy && !after_launch && h->zc_out && h->h_out_dev;
  orbfe_keypoint* o_kps = zc_out ? reinterpret_cast<orbfe_keypoint*>(h->h_out_dev) : h->d_kps;
  uint8_t* o_desc = zc_out ? h->h_out_dev + (h->d_desc - h->d_out) : h->d_desc;
  int32_t* o_counts =
      zc_out ? reinterpret_cast<int32_t*>(h->h_out_dev + (reinterpret_cast<uint8_t*>(h->d_counts) - h->d_out))
             : h->d_counts;
  static const bool trace = std::getenv("ORBFE_HOST_TRACE") != nullptr;  // phase times to stderr
  auto now = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = trace ? now() : 0.0;
  auto part = [n](int c, int parts) { return (int)((long long)c * n / parts); };
  for (int g = 0; g < ngroups; g++) {
    for (int c = g * cpg; c < (g + 1) * cpg; c++) {
      const int i0 = part(c, nchunks), nc = part(c + 1, nchunks) - i0;
      if (direct_in) {  // one DMA per run of images adjacent in the caller's memory
        for (int i = i0; i < i0 + nc;) {
          int j = i + 1;
          while (j < i0 + nc && imgs[j] == imgs[j - 1] + img_bytes) j++;
          ORBFE_HIP_CHECK(hipMemcpyAsync(h->d_in + (size_t)i * img_bytes, imgs[i], (size_t)(j - i) * img_bytes,
                                         hipMemcpyHostToDevice, s_in));
          i = j;
        }
        continue;
      }
      auto stage = [&](int task) {
        const int i = i0 + task / bands, r0 = (task % bands) * band, r1 = std::min(rows, r0 + band);
        if (zc_l0) {  // the level-0 layout: 4 bytes before column 0, REFLECT_101 columns -3..-1, w..w+2
          const int P = h->levels[0].pitch, w = cols;
          for (int r = r0; r < r1; r++) {
            const uint8_t* srow = imgs[i] + (size_t)r * step;
            uint8_t* row = h->h_in + (size_t)i * l0_bytes + (size_t)r * P + 4;
            std::memcpy(row, srow, cols);
            row[-1] = srow[1];
            row[-2] = srow[2];
            row[-3] = srow[3];
            row[w] = srow[w - 2];
            row[w + 1] = srow[w - 3];
            row[w + 2] = srow[w - 4];
          }
          return;
        }
        uint8_t* dst = h->h_in + (size_t)i * img_bytes;
        if (step == (size_t)cols) {
          std::memcpy(dst + (size_t)r0 * cols, imgs[i] + (size_t)r0 * cols, (size_t)(r1 - r0) * cols);
        } else {
          for (int r = r0; r < r1; r++) std::memcpy(dst + (size_t)r * cols, imgs[i] + (size_t)r * step, cols);
        }
      };
      if ((size_t)nc * img_bytes >= ((size_t)2 << 20)) {
        h->pool->parallel_for(nc * bands, stage);
      } else {  // a small chunk (a single image): the workers' wake-up costs more than the copy
        for (int task = 0; task < nc * bands; task++) stage(task);
      }
      if (zc_in) continue;  // k_copy0 reads the staging buffer itself
      ORBFE_HIP_CHECK(hipMemcpyAsync(h->d_in + (size_t)i0 * img_bytes, h->h_in + (size_t)i0 * img_bytes,
                                     (size_t)nc * img_bytes, hipMemcpyHostToDevice, s_in));
    }
    const int g0 = part(g, ngroups), ng = part(g + 1, ngroups) - g0;
    if (trace) std::fprintf(stderr, "[host] group %d staged + H2D enqueued %.1f\n", g, now() - t_start);
    if (!small) {
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_in[g], h->h2d));
      ORBFE_HIP_CHECK(hipStreamWaitEvent(h->stream, h->ev_in[g], 0));
    }
    h->input_l0 = zc_l0;
    st = launch_extract_graphed(h, ng, zc_in ? h->h_in_dev + (size_t)g0 * l0_bytes : h->d_in + (size_t)g0 * img_bytes,
                                zc_in ? (long long)l0_bytes : (long long)img_bytes, zc_l0 ? h->levels[0].pitch : cols,
                                o_kps + (size_t)g0 * K, o_desc + (size_t)g0 * K * 32, K, o_counts + g0,
                                h->stream, g0);
    h->input_l0 = false;
    if (st != ORBFE_OK) return st;
    if (trace) std::fprintf(stderr, "[host] group %d launched %.1f\n", g, now() - t_start);
    if (after_launch) {  // (small: one group on the handle's stream, before the results' copies)
      st = after_launch();
      if (st != ORBFE_OK) return st;
    }
    if (h->host_pyramid) {
      // mvImagePyramid for a CPU Frame::ComputeStereoMatches: the group's pyramids go down on the
      // second copy stream as soon as they are built, beside FAST / DistributeOctTree / describe
      ORBFE_HIP_CHECK(hipStreamWaitEvent(h->d2h, h->ev_pyr, 0));
      ORBFE_HIP_CHECK(hipMemcpyAsync(h->h_pyr + (size_t)g0 * h->pyr_stride, h->d_pyr + (size_t)g0 * h->pyr_stride,
                                     (size_t)ng * h->pyr_stride, hipMemcpyDeviceToHost, h->d2h));
      for (int i = g0; i < g0 + ng; i++) h->h_pyr_gen[i] = h->gen;
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_hpyr, h->d2h));
      h->hpyr_pending = true;
    }
    if (!small) {
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_ext[g], h->stream));
      ORBFE_HIP_CHECK(hipStreamWaitEvent(h->d2h, h->ev_ext[g], 0));
    }
    if (zc_out) {  // the results are in h_out once the stream gets here
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_out[0], s_out));
      continue;
    }
    if (one_copy) {  // (small: one group, one piece)
      const size_t span = (reinterpret_cast<uint8_t*>(h->d_counts) - h->d_out) + sizeof(int32_t) * (size_t)n;
      ORBFE_HIP_CHECK(hipMemcpyAsync(h->h_out, h->d_out, span, hipMemcpyDeviceToHost, s_out));
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_out[0], s_out));
      if (trace) std::fprintf(stderr, "[host] group %d D2H enqueued %.1f\n", g, now() - t_start);
      continue;
    }
    ORBFE_HIP_CHECK(hipMemcpyAsync(hc + g0, h->d_counts + g0, sizeof(int32_t) * ng, hipMemcpyDeviceToHost, s_out));
    const int ppg = npieces / ngroups;
    for (int p = ppg * g; p < ppg * (g + 1); p++) {
      const int i0 = part(p, npieces), np = part(p + 1, npieces) - i0;
      orbfe_keypoint* kd = direct_out ? kps : hk;  // cap == K on the direct path
      uint8_t* dd = direct_out ? desc : hd;
      ORBFE_HIP_CHECK(hipMemcpyAsync(kd + (size_t)i0 * K, h->d_kps + (size_t)i0 * K, (size_t)np * K * sizeof(orbfe_keypoint),
                                     hipMemcpyDeviceToHost, s_out));
      ORBFE_HIP_CHECK(hipMemcpyAsync(dd + (size_t)i0 * K * 32, h->d_desc + (size_t)i0 * K * 32, (size_t)np * K * 32,
                                     hipMemcpyDeviceToHost, s_out));
      ORBFE_HIP_CHECK(hipEventRecord(h->ev_out[p], s_out));
    }
    if (trace) std::fprintf(stderr, "[host] group %d staged + enqueued %.1f\n", g, now() - t_start);
  }
  int need = 0;
  for (int p = 0; p < npieces; p++) {
    const int i0 = part(p, npieces), np = part(p + 1, npieces) - i0;
    ORBFE_HIP_CHECK(hipEventSynchronize(h->ev_out[p]));
    if (trace) std::fprintf(stderr, "[host] piece %d arrived %.1f\n", p, now() - t_start);
    for (int i = i0; i < i0 + np; i++) {  // (a piece's counts arrived before its slots)
      counts[i] = hc[i];
      need = std::max(need, (int)hc[i]);
    }
    if (need > cap || (need > 0 && !per_image && (!kps || !desc))) break;  // reported below
    if (direct_out) continue;  // the slots landed in the caller's buffers
    auto unpack = [&](int k) {
      const int i = i0 + k;
      if (hc[i] == 0) return;
      std::memcpy(per_image ? kps_img[i] : kps + (size_t)i * cap, hk + (size_t)i * K, sizeof(orbfe_keypoint) * hc[i]);
      std::memcpy(per_image ? desc_img[i] : desc + (size_t)i * cap * 32, hd + (size_t)i * K * 32, (size_t)32 * hc[i]);
    };
    h->pool->parallel_for(np, unpack);
  }
  if (need > cap || (need > 0 && !per_image && (!kps || !desc))) ORBFE_HIP_CHECK(hipStreamSynchronize(s_out));
  if (trace) std::fprintf(stderr, "[host] done %.1f\n", now() - t_start);
  h->call_inline = false;
  if (tune_arm >= 0) {
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call).count();
    (tune_arm ? tune->t_one : tune->t_two).push_back(us);
    if (tune->t_one.size() >= 6 && tune->t_two.size() >= 6) {
      auto trimmed_mean = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        double sum = 0;
        for (size_t i = 0; i + 1 < v.size(); i++) sum += v[i];
        return sum / (double)(v.size() - 1);
      };
      tune->decided = trimmed_mean(tune->t_one) < 0.9 * trimmed_mean(tune->t_two) ? 1 : 0;
    }
  }
  if (need > cap) return orbfe_set_error(ORBFE_ERR_CAPACITY, "keypoint capacity too small");
  if (need > 0 && !per_image && (!kps || !desc)) return orbfe_set_error(ORBFE_ERR_ARG, "null output buffer");
  return ORBFE_OK;
}

extern "C" int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int rows, int cols,
                             size_t step, orbfe_keypoint* kps, int cap, uint8_t* desc, int* n) {
  if (!n) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extract: n is NULL");
  *n = 0;
  if (rows == 0 || cols == 0) return ORBFE_OK;
  int32_t cnt = 0;
  const uint8_t* imgs[1] = {img};
  const int st = orbfe_extract_batch(h, 1, imgs, rows, cols, step, kps, desc, cap, &cnt);
  *n = cnt;
  return st;
}

extern "C" int orbfe_get_level_device(orbfe_extractor* h, int image, int level,
                                      const uint8_t** d_p, int* rows, int* cols, size_t* step) {
  if (!h || !d_p || !rows || !cols || !step) return ORBFE_ERR_ARG;
  if (!h->last_img0 || image < 0 || image >= h->last_n || level < 0 || level >= h->nlevels)
    return orbfe_set_error(ORBFE_ERR_STATE, "orbfe_get_level: no such image/level in the last call");
  const LevelDesc& d = h->levels[level];
  *rows = d.h;
  *cols = d.w;
  *d_p = h->d_pyr + (long long)image * h->pyr_stride + d.pyr_off;
  *step = (size_t)d.pitch;
  return ORBFE_OK;
}

int orbfe_internal_pyramid(orbfe_extractor* h, OrbfePyramid* out) {
  if (!h || !out) return ORBFE_ERR_ARG;
  if (!h->last_img0 || h->last_n <= 0)
    return orbfe_set_error(ORBFE_ERR_STATE, "no extract call on this handle yet");
  if (h->nlevels > ORBFE_MAX_LEVELS) return orbfe_set_error(ORBFE_ERR_ARG, "too many levels");
  out->base = h->d_pyr;
  out->image_stride = h->pyr_stride;
  out->n_images = h->last_n;
  out->nlevels = h->nlevels;
  for (int l = 0; l < h->nlevels; l++) {
    const LevelDesc& d = h->levels[l];
    out->w[l] = d.w;
    out->h[l] = d.h;
    out->pitch[l] = d.pitch;
    out->off[l] = d.pyr_off;
    out->scale[l] = h->scale[l];
    out->inv_scale[l] = h->inv_scale[l];
  }
  out->total_key_slots = h->total_key_slots;
  out->io_kps = h->d_kps;
  out->io_desc = h->d_desc;
  out->io_counts = h->d_counts;
  out->stream = h->stream;
  out->device = h->device;
  return ORBFE_OK;
}

OrbfeStereoScratch** orbfe_internal_stereo_slot(orbfe_extractor* h) { return &h->stereo; }

extern "C" int orbfe_get_level(orbfe_extractor* h, int image, int level, const uint8_t** p,
                               int* rows, int* cols, size_t* step) {
  if (!p) return ORBFE_ERR_ARG;
  const uint8_t* dp = nullptr;
  size_t dstep = 0;
  int st = orbfe_get_level_device(h, image, level, &dp, rows, cols, &dstep);
  if (st != ORBFE_OK) return st;
  hipSetDevice(h->device);
  if (h->hpyr_pending) {  // the prefetch copies of the last host-buffer call
    ORBFE_HIP_CHECK(hipEventSynchronize(h->ev_hpyr));
    h->hpyr_pending = false;
  }
  if ((int)h->h_pyr_gen.size() <= image || h->h_pyr_gen[image] != h->gen) {
    // first access to this image since the extract call: copy its whole pyramid (every level, one
    // DMA) once the call's work on its stream is done. The block is sized for all the call's
    // images up front, so the levels handed out before stay where they are.
    bool fresh = true;
    for (int i = 0; i < (int)h->h_pyr_gen.size() && fresh; i++) fresh = h->h_pyr_gen[i] != h->gen;
    if (fresh) {
      st = ensure_host_pyramid(h, h->last_n);
      if (st != ORBFE_OK) return st;
    }
    const hipStream_t s = h->last_stream ? h->last_stream : h->stream;
    ORBFE_HIP_CHECK(hipMemcpyAsync(h->h_pyr + (size_t)image * h->pyr_stride, h->d_pyr + (size_t)image * h->pyr_stride,
                                   (size_t)h->pyr_stride, hipMemcpyDeviceToHost, s));
    ORBFE_HIP_CHECK(hipStreamSynchronize(s));
    h->h_pyr_gen[image] = h->gen;
  }
  const LevelDesc& d = h->levels[level];
  *p = h->h_pyr + (size_t)image * h->pyr_stride + d.pyr_off;
  *step = (size_t)d.pitch;
  return ORBFE_OK;
}

// profiling builds only (not declared in a header): the k_octree phase clocks, 64 * 16 * 16 values
extern "C" int orbfe_debug_octree_prof(unsigned long long* out, int cap) {
#ifdef ORBFE_OCT_PROF
  if (!out || cap < 64 * 16 * 16) return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oct_prof), sizeof(unsigned long long) * 64 * 16 * 16));
  return ORBFE_OK;
#else
  (void)out;
  (void)cap;
  return orbfe_set_error(ORBFE_ERR_STATE, "built without ORBFE_OCT_PROF");
#endif
}

extern "C" int orbfe_extractor_set_graphs(orbfe_extractor* h, int enable) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extractor_set_graphs: null handle");
  hipSetDevice(h->device);
  if (!enable) drop_graphs(h);
  h->use_graphs = enable ? 1 : 0;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_graph_stats(const orbfe_extractor* h, long long* out3) {
  if (!h || !out3) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_graph_stats: bad argument");
  out3[0] = (long long)h->graph_captures;
  out3[1] = (long long)h->graph_hits;
  out3[2] = (long long)h->graphs.size();
  return ORBFE_OK;
}

extern "C" int orbfe_extractor_set_host_pyramid(orbfe_extractor* h, int enable) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_extractor_set_host_pyramid: null handle");
  h->host_pyramid = enable ? 1 : 0;
  return ORBFE_OK;
}

// ---------------------------------------------------------------------------------------------
// stage inspection for per-stage parity tests (orbfe_debug.h)
extern "C" int orbfe_debug_get_candidates(orbfe_extractor* h, int image, int level, uint32_t* out,
                                          int cap, int* n) {
  if (!h || !n || image < 0 || image >= h->last_n || level < 0 || level >= h->nlevels)
    return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipStreamSynchronize(h->stream));
  const LevelDesc& d = h->levels[level];
  std::vector<int32_t> cnt(d.ncells);
  ORBFE_HIP_CHECK(hipMemcpy(cnt.data(), h->d_cellcnt + (size_t)image * h->cells.size() + d.cell_begin,
                            sizeof(int32_t) * d.ncells, hipMemcpyDeviceToHost));
  std::vector<uint32_t> cand(d.cand_cap);
  if (d.cand_cap)
    ORBFE_HIP_CHECK(hipMemcpy(cand.data(), h->d_cand + (size_t)image * h->cand_stride + d.cand_begin,
                              sizeof(uint32_t) * d.cand_cap, hipMemcpyDeviceToHost));
  int tot = 0;
  for (int c = 0; c < d.ncells; c++) {
    const CellDesc& cd = h->cells[d.cell_begin + c];
    for (int i = 0; i < cnt[c]; i++) {
      if (out && tot < cap) out[tot] = cand[cd.slot - d.cand_begin + i];
      tot++;
    }
  }
  *n = tot;
  return (out && tot > cap) ? ORBFE_ERR_CAPACITY : ORBFE_OK;
}

extern "C" int orbfe_debug_candidate_total(orbfe_extractor* h, long long* total) {
  if (!h || !total || h->last_n <= 0) return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipStreamSynchronize(h->stream));
  std::vector<int32_t> cnt((size_t)h->last_n * h->cells.size());
  ORBFE_HIP_CHECK(hipMemcpy(cnt.data(), h->d_cellcnt, sizeof(int32_t) * cnt.size(), hipMemcpyDeviceToHost));
  long long t = 0;
  for (int32_t c : cnt) t += c;
  *total = t;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_get_level_keys(orbfe_extractor* h, int image, int level,
                                          uint32_t* out, int cap, int* n) {
  if (!h || !n || image < 0 || image >= h->last_n || level < 0 || level >= h->nlevels)
    return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipStreamSynchronize(h->stream));
  int32_t cnt = 0;
  ORBFE_HIP_CHECK(hipMemcpy(&cnt, h->d_lvlcnt + (size_t)image * h->nlevels + level, sizeof(int32_t),
                            hipMemcpyDeviceToHost));
  *n = cnt;
  if (!out) return ORBFE_OK;
  if (cnt > cap) return ORBFE_ERR_CAPACITY;
  if (cnt > 0)
    ORBFE_HIP_CHECK(hipMemcpy(out, h->d_lvlkeys + (size_t)image * h->lvlkey_stride + h->levels[level].key_begin,
                              sizeof(uint32_t) * cnt, hipMemcpyDeviceToHost));
  return ORBFE_OK;
}

extern "C" int orbfe_debug_get_blurred(orbfe_extractor* h, int image, int level, uint8_t* out,
                                       int cap) {
  if (!h || !out || image < 0 || image >= h->last_n || level < 0 || level >= h->nlevels)
    return ORBFE_ERR_ARG;
  const LevelDesc& d = h->levels[level];
  if (cap < d.w * d.h) return ORBFE_ERR_CAPACITY;
  ORBFE_HIP_CHECK(hipStreamSynchronize(h->stream));
  ORBFE_HIP_CHECK(hipMemcpy2D(out, d.w, h->d_blur + (size_t)image * h->pyr_stride + d.pyr_off, d.pitch,
                              d.w, d.h, hipMemcpyDeviceToHost));
  return ORBFE_OK;
}

extern "C" int orbfe_debug_steer_trig(uint32_t deg_bits_begin, uint32_t n, float* d_cos, float* d_sin,
                                      void* stream) {
  if (n > 0 && (!d_cos || !d_sin)) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_steer_trig: bad argument");
  hipStream_t st = (hipStream_t)stream;
  if (n > 0)
    hipLaunchKernelGGL(k_steer_trig, dim3((n + 255) / 256), dim3(256), 0, st, deg_bits_begin, n,
                       (float)(M_PI / 180.f), d_cos, d_sin);
  ORBFE_HIP_CHECK(hipGetLastError());
  ORBFE_HIP_CHECK(hipStreamSynchronize(st));
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_blur_mode(orbfe_extractor* h, int mode) {
  if (!h || mode < 0 || mode > 1) return ORBFE_ERR_ARG;
  h->blur_mode = mode;
  return ORBFE_OK;
}

extern "C" int orbfe_set_side_stream(orbfe_extractor* h, void* stream) {
  if (!h) return ORBFE_ERR_ARG;
  h->side_ext = (hipStream_t)stream;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_inline_side(orbfe_extractor* h, int on) {
  if (!h) return ORBFE_ERR_ARG;
  h->inline_side = on ? 1 : 0;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_fast_wpb(orbfe_extractor* h, int side_wpb, int main_wpb) {
  auto ok = [](int v) { return v == 1 || v == 2 || v == 4 || v == 8; };
  if (!h || !ok(side_wpb) || !ok(main_wpb))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_fast_wpb: 1, 2, 4 or 8 cells per workgroup");
  h->fast_wpb_side = side_wpb;
  h->fast_wpb_main = main_wpb;
  drop_graphs(h);
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_lds(orbfe_extractor* h, int hi_kb, int lo_kb) {
  if (!h || hi_kb < 16 || hi_kb > 160 || lo_kb < 16 || lo_kb > 160)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_octree_lds: budgets must be 16-160 KiB");
  h->oct_hi_kb = hi_kb;
  h->oct_lo_kb = lo_kb;
  h->rows = h->cols = -1;  // the LDS plans follow on the next call's geometry
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_split(orbfe_extractor* h, int k) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_octree_split: null handle");
  h->octree_split = k > 0 ? k : 0;
  h->rows = h->cols = -1;  // the LDS plans follow on the next call's geometry
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_fast_side_merge(orbfe_extractor* h, int merge) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_fast_side_merge: null handle");
  h->fast_side_merge = merge ? 1 : 0;
  drop_graphs(h);
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_schedule_autotune(orbfe_extractor* h, int enable) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_schedule_autotune: null handle");
  h->autotune = enable ? 1 : 0;
  for (auto& t : h->tune) t = orbfe_extractor::SchedTune();
  return ORBFE_OK;
}

extern "C" int orbfe_debug_schedule_choice(const orbfe_extractor* h, int n_images) {
  if (!h || n_images < 1 || n_images > 7) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_schedule_choice: bad argument");
  return h->tune[n_images].decided;
}

extern "C" int orbfe_debug_set_zero_copy(orbfe_extractor* h, int input, int output) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_zero_copy: null handle");
  h->zc_in = input == 2 ? 2 : input ? 1 : 0;
  h->zc_out = output ? 1 : 0;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_pyramid_tiles(orbfe_extractor* h, int small_tx, int small_ty, int batch_tx,
                                             int batch_ty) {
  auto ok = [](int x, int y) { return (x == 0 && y == 0) || (x > 0 && y > 0 && x * y <= 4096); };
  if (!h || !ok(small_tx, small_ty) || !ok(batch_tx, batch_ty))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_pyramid_tiles: 0 x 0 or a positive tiling");
  h->pyr_tiles_small[0] = small_tx;
  h->pyr_tiles_small[1] = small_ty;
  h->pyr_tiles_batch[0] = batch_tx;
  h->pyr_tiles_batch[1] = batch_ty;
  h->rows = h->cols = -1;  // the tile plans follow on the next call's geometry
  drop_graphs(h);
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_threads(orbfe_extractor* h, int small_calls, int batches) {
  auto ok = [](int t) { return t == 256 || t == 512 || t == 1024; };
  if (!h || !ok(small_calls) || !ok(batches))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_octree_threads: 256, 512 or 1024");
  h->oct_threads_small = small_calls;
  h->oct_threads_batch = batches;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_threads_l0(orbfe_extractor* h, int threads) {
  if (!h || !(threads == 0 || threads == 256 || threads == 512 || threads == 1024))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_octree_threads_l0: 0, 256, 512 or 1024");
  h->oct_threads_l0 = threads;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_serial(orbfe_extractor* h, int small_calls, int batches) {
  if (!h || small_calls < 1 || small_calls > OCT_SMALL_MAX || batches < 1 || batches > OCT_SMALL_MAX)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_octree_serial: 1 .. 128 keys");
  h->oct_small_small = small_calls;
  h->oct_small_batch = batches;
  drop_graphs(h);  // (the captured launches hold the old value)
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_latency_schedule(orbfe_extractor* h, int k) {
  if (!h) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_debug_set_latency_schedule: null handle");
  h->lat_sched = k > 0 ? k : 0;
  drop_graphs(h);  // a captured sequence follows the old schedule
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_fast_side_levels(orbfe_extractor* h, int k) {
  if (!h) return ORBFE_ERR_ARG;
  h->fast_side_levels = k > 0 ? k : -1;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_get_umax(const orbfe_extractor* h, int32_t* umax16) {
  if (!h || !umax16) return ORBFE_ERR_ARG;
  for (int v = 0; v < 16; v++) umax16[v] = h->umax[v];
  return ORBFE_OK;
}

extern "C" int orbfe_debug_set_octree_key_cap(orbfe_extractor* h, int cap) {
  if (!h) return ORBFE_ERR_ARG;
  h->octree_key_cap_override = cap < 0 ? -1 : (cap & ~63);
  h->rows = h->cols = -1;  // recompute the geometry on the next call
  return ORBFE_OK;
}

extern "C" int orbfe_debug_geometry(orbfe_extractor* h, int rows, int cols, int32_t* info, int cap) {
  // per level: w, h, ncells, cand_cap, budget, nini, key_cap (7 ints)
  if (!h || !info) return ORBFE_ERR_ARG;
  hipSetDevice(h->device);
  const int st = compute_geometry(h, rows, cols);
  if (st != ORBFE_OK) return st;
  if (cap < 7 * h->nlevels) return ORBFE_ERR_CAPACITY;
  for (int l = 0; l < h->nlevels; l++) {
    const LevelDesc& d = h->levels[l];
    int32_t* o = info + 7 * l;
    o[0] = d.w;
    o[1] = d.h;
    o[2] = d.ncells;
    o[3] = d.cand_cap;
    o[4] = d.budget;
    o[5] = d.nini;
    o[6] = d.key_cap;
  }
  return ORBFE_OK;
}
