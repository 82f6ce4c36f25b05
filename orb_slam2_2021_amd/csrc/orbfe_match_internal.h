// orbfe_match_internal.h -- library-internal pieces of the matcher shared by orbfe_match.hip (the
// SearchByProjection engine, SearchForTriangulation, isInFrustum), orbfe_project.hip (the
// keyframe / loop-closing projection searches) and orbfe_bow.hip (SearchByBoW,
// SearchForInitialization, ComputeDistinctiveDescriptors). Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cstring>
#include <tuple>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_match_batch.h"
#include "orbfe_device.h"

#define TH_HIGH 100
#define TH_LOW 50
#define HISTO_LENGTH 30
#define GRID_COLS 64
#define GRID_ROWS 48
#define GRID_CELLS (GRID_COLS * GRID_ROWS)
#define SBP_MAX_ROUNDS 12      // rounds of the first launch (no host sync)
#define SBP_ROUND_CAP 1024     // rounds a host-synchronous search may continue to before the serial walk
#define SBP_FINAL_SLOT (SBP_ROUND_CAP + 3)  // state[]: 1 + the result buffer k_sbp_settle left final (0: by parity)
#define GRID_MAX_KEYS 8192   // frame keypoints per matcher call (k_grid sorts them in LDS)
#define SFT_MAX_KF2 16384    // KF2 keypoints per SearchForTriangulation pair (claim bitmap)
#define SBP_CAND 48          // default per-query candidate cache of the projection searches
#define SWEEP_THREADS 1024   // k_sbp_sweep: one workgroup walks the claim order chunk by chunk
#define SWEEP_MAX_KEYS 4096  // frame keypoints k_sbp_sweep keeps owners of in LDS (more: grid rounds)
#define ORBFE_MAX_LEVELS_M 32

struct orbfe_matcher {
  int device = 0;
  float nnratio;
  int check_ori;
  hipStream_t stream = nullptr;
  // device arena (grown on demand)
  uint8_t* arena = nullptr;
  size_t arena_bytes = 0;
  orbfe_sft_pair* d_pairs = nullptr;
  int pairs_cap = 0;
  std::vector<orbfe_sft_pair> pairs_uploaded;  // host copy of d_pairs (skip identical uploads)
  int32_t* d_serial = nullptr;
  // pinned mirror of the arena: host inputs are staged at their arena offsets and uploaded in one
  // H2D copy per call instead of one pageable copy per array
  uint8_t* pinned = nullptr;
  size_t pinned_bytes = 0;
  size_t stage_lo = SIZE_MAX, stage_hi = 0;
  // inputs the caller passed in device memory: arena offset, source, bytes; copied on the device
  // after the staged span's H2D copy (which may cover their arena regions)
  std::vector<std::tuple<size_t, const void*, size_t>> d2d;
  // results wanted on the host: caller destination, arena offset, bytes (fetch_d2h takes them down
  // through the pinned mirror, one copy when their span is small)
  std::vector<std::tuple<void*, size_t, size_t>> d2h;
  int last_rounds = 0, last_serial = 0;
  bool sbp_deferred = false;  // the last SearchByProjection launch left its rounds to the host (sbp_fetch)
  bool sbp_swept = false;     // ... and whether k_sbp_sweep settled its claim order
  int max_rounds = SBP_MAX_ROUNDS;
  int round_cap = SBP_ROUND_CAP;  // >= max_rounds; equal: no continuation (serial fallback at once)
  // orbfe_debug_matcher_set_sweep (0: the defaults): queries per k_sbp_sweep chunk, Jacobi rounds a
  // chunk may take before its sequential walk, cache entries per query (SBP_CAND)
  int sweep_chunk = 0, sweep_max_rounds = 0, cand_cap = 0;
  // k_sbp_sweep's dynamic-LDS limit on this matcher's device: 0 not set yet, 1 set, -1 refused
  // (the sweep is then off for this matcher)
  int sweep_attr = 0;
  // orbfe_matcher_set_profiling: HIP events around the device part (first kernel .. last kernel,
  // no H2D / D2H) of each SearchByProjection-family call
  int profile = 0;
  bool prof_started = false, prof_done = false;
  hipError_t pending_err = hipSuccess;  // found by stage_h2d's pointer query, reported by flush_h2d
  hipEvent_t prof_ev0 = nullptr, prof_ev1 = nullptr;
};

// device-time window of one call (orbfe_matcher_set_profiling)
inline void prof_begin(orbfe_matcher* m) {
  if (m->profile && !m->prof_started) {
    hipEventRecord(m->prof_ev0, m->stream);
    m->prof_started = true;
  }
}
inline void prof_end(orbfe_matcher* m) {
  if (m->profile && m->prof_started && !m->prof_done) {
    hipEventRecord(m->prof_ev1, m->stream);
    m->prof_done = true;
  }
}

// SearchByProjection's per-query candidate cache entry: keypoint index | Hamming distance << 16 |
// octave << 24 (one dword per candidate; a distance of 256 is never cached)
__host__ __device__ __forceinline__ uint32_t cand_pack(int k, int dist, int level) {
  return (uint32_t)k | ((uint32_t)dist << 16) | ((uint32_t)level << 24);
}
__host__ __device__ __forceinline__ int cand_key(uint32_t e) { return (int)(e & 0xffffu); }
__host__ __device__ __forceinline__ int cand_dist(uint32_t e) { return (int)((e >> 16) & 0xffu); }
__host__ __device__ __forceinline__ int cand_level(uint32_t e) { return (int)(e >> 24); }

// ---- device helpers shared by the matcher kernels ---------------------------------------------
__device__ __forceinline__ int rot_bin_dev(float a1, float a2) {
  // ORBmatcher.cc:781-786 (only bins 0..12 are reachable: round(rot * 1/30); kept as is)
  const float factor = 1.0f / HISTO_LENGTH;
  float rot = a1 - a2;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)roundf(rot * factor);
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

// ComputeThreeMaxima (ORBmatcher.cc:1627-1668) on 30 counts
__device__ __forceinline__ void three_maxima_dev(const int* h, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < HISTO_LENGTH; i++) {
    const int s = h[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s; ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
  else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

// cv::Mat CV_32F 3x3 gemm row: double accumulation, one rounding
__device__ __forceinline__ float gemv3_d(const float* r, float x, float y, float z, float add) {
  double s = (double)r[0] * (double)x;
  s += (double)r[1] * (double)y;
  s += (double)r[2] * (double)z;
  s = s + (double)add;
  return (float)s;
}

// MapPoint::PredictScale (MapPoint.cc:415-447) from the host-built threshold table
// (orbfe_predict_scale_thresholds): #{k : ratio >= thr[k-1]}.
__device__ __forceinline__ int predict_scale_dev(float max_distance, float dist, const float* thr,
                                                 int nlevels) {
  const float ratio = max_distance / dist;
  int s = 0;
  for (int k = 1; k < nlevels; k++) s += ratio >= thr[k - 1] ? 1 : 0;
  return s;
}

// ---- SearchByProjection engine (orbfe_match.hip) -----------------------------------------------
// gate: how a window candidate's stereo coordinate is tested before its distance is computed
#define SBP_GATE_STEREO 0  // uRight > 0 and |xr - uRight| > er_lim rejects (:95-100, :1429-1436)
#define SBP_GATE_NONE 1
#define SBP_GATE_FUSE 2    // Fuse's reprojection error test with (x, y, xr) = (u, v, ur) (:930-954)

struct SbpQuery {
  float x, y, r;      // search window centre and half-size (GetFeaturesInArea's x, y, r)
  float xr, er_lim;   // stereo coordinate of the projection; stereo-gate limit
  int min_level, max_level;
  int flags;          // bit0 valid query, bit1 an assignment blocks the keypoint for later queries
  int gate;           // SBP_GATE_*
};

#define SBP_BLOCK_OBSERVED 0  // mp_state == ORBFE_MP_OBSERVED (Observations() > 0: :91-93, :1420-1422)
#define SBP_BLOCK_ANY 1       // mp_state != ORBFE_MP_NONE (any non-NULL entry: :384, :1567)
#define SBP_BLOCK_NONE 2      // nothing (Fuse, SearchBySim3 never skip a keypoint)

struct SbpMode {
  int mode;       // 0 best + second + ratio (local map), 1 first minimum (all other overloads)
  int dist_th;    // accept bestDist <= dist_th
  int block_any;  // SBP_BLOCK_*: which keypoints are taken before the search starts
  int check_ori;  // rotation-consistency filter over q_angle (mode 1)
  int no_claims;  // 1: no assignment blocks a keypoint (Fuse, SearchBySim3): one round suffices
};

namespace orbfe_mi {
struct Arena {
  size_t total = 0;
  size_t add(size_t bytes) {
    const size_t off = total;
    total += (bytes + 255) & ~(size_t)255;
    return off;
  }
};
int ensure_arena(orbfe_matcher* m, size_t bytes);
void stage_h2d(orbfe_matcher* m, const void* dst, const void* src, size_t n);
int flush_h2d(orbfe_matcher* m);
// Queue `n` bytes of arena address `src` for the host address `dst`; fetch_d2h copies every queued
// region down (one copy of their span into the pinned mirror when it is at most 4x their bytes plus
// 64 KiB, else one copy each), synchronises the matcher's stream and copies them out.
void stage_d2h(orbfe_matcher* m, void* dst, const void* src, size_t n);
int fetch_d2h(orbfe_matcher* m);

struct FrameOffsets {
  size_t keys, ur, desc, mp, scale, sigma2;
};
FrameOffsets plan_frame(Arena& ar, const orbfe_frame_view* f);
int upload_frame(orbfe_matcher* m, const FrameOffsets& o, const orbfe_frame_view* f,
                 orbfe_frame_view* d);
bool frame_ok(const orbfe_frame_view* f);
bool levels_ok(const orbfe_keypoint* k, int n, int nlevels);

// One SearchByProjection-shaped search (queries x frame grid) in the arena.
struct SbpPlan {
  FrameOffsets fo;
  size_t oqd, oqa, og_start, og_items, oq, ores0, ores1, oown0, oown1, oown2, oblk, ostate, obest;
  size_t ocand, ocand_n, onm, oown3, olive;
  bool cache;
  bool sweep;  // the claim order in k_sbp_sweep after round 0 (the candidate cache exists)
  int nq, cand_cap;
};
SbpPlan sbp_plan(Arena& ar, const orbfe_frame_view* F, int nq, int cand_cap = SBP_CAND);
// the two halves of sbp_plan: staged inputs, then device scratch (plan other staged inputs between)
void sbp_plan_inputs(Arena& ar, const orbfe_frame_view* F, int nq, int cand_cap, SbpPlan& p);
// the candidate cache entries per query of matcher m's projection searches (SBP_CAND, or the
// orbfe_debug_matcher_set_sweep override)
int sbp_cand_cap(const orbfe_matcher* m);
void sbp_plan_scratch(Arena& ar, const orbfe_frame_view* F, SbpPlan& p);
// stages the frame and the query descriptors / angles (flush before launching)
int sbp_stage(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const uint8_t* h_qdesc,
              const float* h_qangle, orbfe_frame_view* dF);
// grid, init, fixpoint rounds, collect / finish on the matcher's stream (queries at p.oq)
// With `defer`, a fixpoint still unsettled after the first launch's rounds leaves its results for
// sbp_fetch to continue (more rounds) instead of running the serial walk.
int sbp_launch(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
               const SbpMode& md, bool defer = false);
// D2H of best_idx and the count, stream sync, round statistics. With F / dF / md (a search launched
// with defer), an unsettled fixpoint continues with doubling round chunks up to m->round_cap.
int sbp_fetch(orbfe_matcher* m, const SbpPlan& p, int32_t* best_idx, int* nmatches,
              const orbfe_frame_view* F = nullptr, const orbfe_frame_view* dF = nullptr,
              const SbpMode* md = nullptr);
// grid only (CSR of the frame's keypoints, 16-B records) -- used by SearchForInitialization
void sbp_launch_grid(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF);
// round 0 only (candidate cache + first result), for callers that consume the cache
void sbp_launch_round0(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
                       const SbpMode& md);

// PredictScale thresholds (host logf), see orbfe_predict_scale_thresholds
void predict_scale_table(float log_scale_factor, int nlevels, float* thr);
}  // namespace orbfe_mi
