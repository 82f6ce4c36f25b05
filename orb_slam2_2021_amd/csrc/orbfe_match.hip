// orbfe_match.hip -- ORBmatcher's Hamming searches as CDNA4 kernels (gfx950, wave64).
//
// Reference: src/ORBmatcher.cc of lreithmayr/ORB_SLAM2_2021.
//   SearchForTriangulation (:671-839): keypoints can only pair inside one vocabulary node and every
//     feature sits in exactly one node, so nodes are independent. One wavefront owns a node: lanes
//     hold the KF2 candidates, the KF1 features are walked in order (the reference's claim order,
//     vbMatched2), and each step is one wave-wide min-reduction that returns the LAST candidate at
//     the minimal distance (the reference updates on dist <= bestDist). One workgroup per KF pair;
//     the rotation-consistency histogram (:806-826) runs after a workgroup barrier.
//   SearchByProjection, local map (:45-133) and last frame (:1348-1491): a keypoint taken by an
//     earlier MapPoint with Observations() > 0 is skipped by every later MapPoint. Solved as a
//     parallel fixpoint: round r computes every MapPoint's match against the owners found in round
//     r-1 (owner(k) = lowest MapPoint index claiming k); the first round whose results equal the
//     previous round's is the reference's sequential result (proof in DESIGN.md). Rounds run
//     back-to-back without host syncs; a serial kernel finishes the job if the round budget ran out.
//   Frame::AssignFeaturesToGrid / GetFeaturesInArea (Frame.cc:279-294, 376-445): the 64x48 grid is
//     rebuilt on the device as CSR (bitonic sort of cell<<16 | index keys), and candidates are
//     visited in the reference's order (ix outer, iy inner, ascending index inside a cell).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_frustum.h"
#include "../../include/orbfe_keyframe.h"
#include "../../include/orbfe_match_batch.h"
#include "orbfe_device.h"
#include "orbfe_match_internal.h"
#include "orbfe_ktimer.h"

using namespace orbfe_mi;

// ---------------------------------------------------------------------------------------------
// SearchForTriangulation: k_sft_nodes (one wavefront per KF1 vocabulary node, many workgroups
// per pair; each wavefront writes the final match12 of every KF1 feature of its node, -1 included,
// and one more workgroup per pair writes -1 for the features no node lists, so no initialisation
// pass runs first), k_sft_finish (rotation filter + count per pair).
__device__ __forceinline__ void sft_resolve_sizes(orbfe_sft_pair& P) {
  if (P.kf1_n_dev) P.kf1.n = *P.kf1_n_dev;
  if (P.kf2_n_dev) P.kf2.n = *P.kf2_n_dev;
  if (P.fv1_nodes_dev) P.fv1.n_nodes = *P.fv1_nodes_dev;
  if (P.fv2_nodes_dev) P.fv2.n_nodes = *P.fv2_nodes_dev;
}

#define SFT_REG_CHUNKS 4  // node-2 candidates held in registers: 4 x 64 per wavefront
#define SFT_MAX_NODE (SFT_MAX_KF2)

// Candidate state of one lane for one 64-wide chunk of a node's KF2 features.
struct SftCand {
  uint4 d0, d1;
  float x, y, epi_thr;   // epi_thr = 100 * mvScaleFactors[octave] (:761)
  double sig_thr;        // 3.84 * mvLevelSigma2[octave] (:162)
  int idx2;
  bool usable, stereo;   // usable: in range, no MapPoint, stereo if bOnlyStereo
};

// Per-octave thresholds of KF2, lane l holding octave l (read with a lane shuffle, no dependent
// global load per candidate)
struct SftOctTab {
  float epi;   // 100 * mvScaleFactors[o] (:761)
  double sig;  // 3.84 * mvLevelSigma2[o] (:162)
};
__device__ __forceinline__ SftOctTab sft_oct_tab(const orbfe_sft_pair& P) {
  const int lane = lane_id();
  SftOctTab t;
  t.epi = lane < P.kf2.nlevels ? 100 * P.kf2.scale_factors[lane] : 0.f;
  t.sig = lane < P.kf2.nlevels ? 3.84 * (double)P.kf2.level_sigma2[lane] : 0.0;
  return t;
}

// All of a candidate's loads are issued together (index, then MapPoint state, uRight, keypoint
// and descriptor at once): two dependent rounds.
__device__ __forceinline__ void sft_load_cand(const orbfe_sft_pair& P, int o2, int n2, int p,
                                              int only_stereo, const SftOctTab& tab, SftCand& c) {
  c.usable = false;
  c.stereo = false;
  c.idx2 = -1;
  c.x = c.y = c.epi_thr = 0.f;
  c.sig_thr = 0.0;
  c.d0 = c.d1 = make_uint4(0, 0, 0, 0);
  int oct = 0;
  if (p < n2) {
    const int idx2 = P.fv2.indices[o2 + p];
    const uint8_t mp = P.kf2.mp_state[idx2];
    const float ur = P.kf2.u_right[idx2];
    const orbfe_keypoint kp2 = P.kf2.keys_un[idx2];
    load_desc(P.kf2.descriptors + (size_t)idx2 * 32, c.d0, c.d1);
    c.idx2 = idx2;
    c.stereo = ur >= 0;
    c.usable = mp == ORBFE_MP_NONE && !(only_stereo && !c.stereo);
    c.x = kp2.x;
    c.y = kp2.y;
    oct = kp2.octave;
  }
  c.epi_thr = __shfl(tab.epi, oct, 64);
  c.sig_thr = __shfl(tab.sig, oct, 64);
}

// Key of a passing candidate: smallest distance, then the LAST position (ties replace, :752).
__device__ __forceinline__ unsigned long long sft_key(const SftCand& c, bool claimed, int p,
                                                      const uint4& a0, const uint4& a1, bool st1,
                                                      float ex, float ey, float la, float lb,
                                                      float lc, float den) {
  if (!c.usable || claimed) return ~0ull;
  const int dist = hamming256(a0, a1, c.d0, c.d1);
  if (dist > TH_LOW) return ~0ull;
  if (!st1 && !c.stereo) {
    const float dex = ex - c.x, dey = ey - c.y;
    if (dex * dex + dey * dey < c.epi_thr) return ~0ull;
  }
  if (den == 0) return ~0ull;  // CheckDistEpipolarLine (:153-162)
  const float num = la * c.x + lb * c.y + lc;
  const float dsqr = num * num / den;
  if (!((double)dsqr < c.sig_thr)) return ~0ull;
  return ((unsigned long long)dist << 32) | (unsigned long long)(0x7fffffff - p);
}

// Nodes with at most 64 K features on each side (K = 2: up to SFT_FP_MAX = 128): lanes take KF1
// features (K per lane), every lane finds its passing KF2 candidates once (dist <= TH_LOW, the
// epipole and epipolar checks: the candidate set S_i of the reference loop), then the claim order
// of :772-777 is solved as a fixpoint -- choice(i) = best of S_i minus the choices of features
// before i in the node -- iterated from "no claims" until a round reproduces the previous one.
// That fixpoint is unique and equals the sequential result (feature i's choice is final once
// those before it are).
// (K = 4 for nodes of 129-256 features ran alone in 49 vs ~70 us, but its 44 KiB of LDS per
// workgroup (vs 26 KiB) kept DistributeOctTree's 80 KiB blocks off the CUs it occupied beside the
// extraction: 73.1k vs 78.5k stereo frames/s)
constexpr int SFT_FP_MAX = 128;
template <int K>
__device__ __forceinline__ void sft_node_fixpoint(const orbfe_sft_pair& P, int o1, int n1, int o2, int n2,
                                                  int only_stereo, uint32_t* cdesc, int* claim) {
  const int lane = lane_id();
  // candidates: lane p (and 64 h + p) loads KF2 feature p of the node; descriptors go to LDS
  const SftOctTab tab = sft_oct_tab(P);
  SftCand c[K];
#pragma unroll
  for (int h = 0; h < K; h++) {
    sft_load_cand(P, o2, n2, 64 * h + lane, only_stereo, tab, c[h]);
    if (64 * h + lane < n2) {
      *reinterpret_cast<uint4*>(cdesc + 8 * (64 * h + lane)) = c[h].d0;
      *reinterpret_cast<uint4*>(cdesc + 8 * (64 * h + lane) + 4) = c[h].d1;
    }
  }
  // KF1 features i = 64 k + lane
  int idx1[K];
  bool ok1[K], st1[K];
  float x1[K], y1[K];
  uint4 a0[K], a1[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = 64 * k + lane;
    idx1[k] = -1;
    ok1[k] = false;
    st1[k] = false;
    x1[k] = y1[k] = 0.f;
    a0[k] = a1[k] = make_uint4(0, 0, 0, 0);
    if (i < n1) {
      idx1[k] = P.fv1.indices[o1 + i];
      st1[k] = P.kf1.u_right[idx1[k]] >= 0;
      ok1[k] = P.kf1.mp_state[idx1[k]] == ORBFE_MP_NONE && !(only_stereo && !st1[k]);
      const orbfe_keypoint kp = P.kf1.keys_un[idx1[k]];
      x1[k] = kp.x;
      y1[k] = kp.y;
      load_desc(P.kf1.descriptors + (size_t)idx1[k] * 32, a0[k], a1[k]);
    }
  }
  wave_sync();
  const float* F = P.f12;
  const float f0 = F[0], f1 = F[1], f2 = F[2], f3 = F[3], f4 = F[4], f5 = F[5], f6 = F[6],
              f7 = F[7], f8 = F[8];
  float la[K], lb[K], lc[K], den[K];
#pragma unroll
  for (int k = 0; k < K; k++) {  // epipolar line l = x1' F12 (CheckDistEpipolarLine :149-151)
    la[k] = x1[k] * f0 + y1[k] * f3 + f6;
    lb[k] = x1[k] * f1 + y1[k] * f4 + f7;
    lc[k] = x1[k] * f2 + y1[k] * f5 + f8;
    den[k] = la[k] * la[k] + lb[k] * lb[k];
  }
  // 1. passing sets (bit p - 64 h of pm[k][h] for feature 64 k + lane) and the round-0 choice
  const int kact = (n1 + 63) >> 6;
  uint64_t pm[K][K];
  unsigned long long best[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    best[k] = ~0ull;
#pragma unroll
    for (int h = 0; h < K; h++) pm[k][h] = 0;
  }
#pragma unroll
  for (int h = 0; h < K; h++) {
    const int pend = min(n2, 64 * (h + 1));
    for (int p = 64 * h; p < pend; p++) {
      const int src = p & 63;
      SftCand cb;  // candidate p broadcast from its lane (scalar registers)
      cb.usable = __builtin_amdgcn_readlane((int)c[h].usable, src) != 0;
      if (!cb.usable) continue;  // uniform
      cb.stereo = __builtin_amdgcn_readlane((int)c[h].stereo, src) != 0;
      cb.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c[h].x), src));
      cb.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c[h].y), src));
      cb.epi_thr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c[h].epi_thr), src));
      const long long sb = __double_as_longlong(c[h].sig_thr);
      cb.sig_thr = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(sb >> 32), src) << 32) |
                                        (unsigned)__builtin_amdgcn_readlane((int)(sb & 0xffffffff), src));
      cb.d0.x = __builtin_amdgcn_readlane(c[h].d0.x, src);
      cb.d0.y = __builtin_amdgcn_readlane(c[h].d0.y, src);
      cb.d0.z = __builtin_amdgcn_readlane(c[h].d0.z, src);
      cb.d0.w = __builtin_amdgcn_readlane(c[h].d0.w, src);
      cb.d1.x = __builtin_amdgcn_readlane(c[h].d1.x, src);
      cb.d1.y = __builtin_amdgcn_readlane(c[h].d1.y, src);
      cb.d1.z = __builtin_amdgcn_readlane(c[h].d1.z, src);
      cb.d1.w = __builtin_amdgcn_readlane(c[h].d1.w, src);
      const uint64_t bit = 1ull << src;
#pragma unroll
      for (int k = 0; k < K; k++) {
        if (k < kact && ok1[k]) {  // kact: uniform, skips the chunks no KF1 feature fills
          const unsigned long long key = sft_key(cb, false, p, a0[k], a1[k], st1[k], P.ex, P.ey, la[k], lb[k],
                                                 lc[k], den[k]);
          if (key != ~0ull) {
            pm[k][h] |= bit;
            best[k] = key < best[k] ? key : best[k];
          }
        }
      }
    }
  }
  int ch[K];
#pragma unroll
  for (int k = 0; k < K; k++) ch[k] = best[k] == ~0ull ? -1 : 0x7fffffff - (int)(best[k] & 0xffffffffull);
  // 2. rounds: claim[p] = first feature choosing p; re-choose among the unclaimed-by-earlier
  for (int round = 0; round <= n1; round++) {
    for (int p = lane; p < n2; p += 64) claim[p] = 0x7fffffff;
    wave_sync();
#pragma unroll
    for (int k = 0; k < K; k++)
      if (ch[k] >= 0) atomicMin(&claim[ch[k]], 64 * k + lane);
    wave_sync();
    bool changed = false;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = 64 * k + lane;
      unsigned long long b = ~0ull;
#pragma unroll
      for (int h = 0; h < K; h++) {
        uint64_t m = pm[k][h];
        while (m) {
          const int p = 64 * h + __builtin_ctzll(m);
          m &= m - 1;
          if (claim[p] < i) continue;  // vbMatched2: taken by an earlier feature of the node
          const uint4 d0 = *reinterpret_cast<const uint4*>(cdesc + 8 * p);
          const uint4 d1 = *reinterpret_cast<const uint4*>(cdesc + 8 * p + 4);
          const unsigned long long key = ((unsigned long long)hamming256(a0[k], a1[k], d0, d1) << 32) |
                                         (unsigned long long)(0x7fffffff - p);
          b = key < b ? key : b;
        }
      }
      const int nk = b == ~0ull ? -1 : 0x7fffffff - (int)(b & 0xffffffffull);
      changed = changed || nk != ch[k];
      ch[k] = nk;
    }
    if (wave_ballot(changed) == 0) break;
    wave_sync();  // claim[] is rewritten by the next round
  }
  // every feature of the node gets its final value (-1: no match), written once
#pragma unroll
  for (int k = 0; k < K; k++)
    if (64 * k + lane < n1) P.match12[idx1[k]] = ch[k] >= 0 ? P.fv2.indices[o2 + ch[k]] : -1;
}

// Nodes past 64 features on either side but within SFT_BIG_MAX on both are solved by a whole
// workgroup instead of one wavefront (whose sequential walk of a 133-feature node, ~130 dependent
// claim steps each a wave-wide min, was the kernel's critical path, and whose 2-per-lane fixpoint
// walks a 100-feature node's candidates with two keys per step). SFT_BIG_WG extra workgroups per
// pair find the pair's big nodes (a thread per node, the same common-node lookup the wavefronts
// do) and take every SFT_BIG_WG-th in node order. Per node: thread p stages KF2 candidate p in
// LDS; KF1 feature i is taken by lane i % 64 of one wavefront, or of two when n1 <= 128 (each then
// walks every other candidate, and the halves' passing bits and best keys are merged through LDS),
// for its passing set S_i (a bit mask) and its round-0 choice; then the claim order (:772-777) as
// the same fixpoint as sft_node_fixpoint -- choice(i) = best of S_i minus the choices of the
// features before i -- with claim[p] = atomicMin over the choosers and a workgroup vote per round.
// The node's LDS (15.9 KiB) aliases the wavefronts' 18 KiB, so the kernel's LDS does not grow.
constexpr int SFT_BIG_MAX = 256;
constexpr int SFT_BIG_WG = 2;
constexpr int SFT_LDS_BYTES = 4 * (SFT_FP_MAX * 8 * 4 + SFT_FP_MAX * 4);  // 18 KiB
__device__ __forceinline__ bool sft_big_node(int n1, int n2) {
  return (n1 > 64 || n2 > 64) && n1 <= SFT_BIG_MAX && n2 <= SFT_BIG_MAX;
}
struct SftBigLds {
  uint4 desc[SFT_BIG_MAX][2];  // candidate descriptors (8 KiB)
  float4 xye[SFT_BIG_MAX];     // x, y, 100 * scale[octave] (4 KiB)
  double sig[SFT_BIG_MAX];     // 3.84 * sigma2[octave] (2 KiB)
  int claim[SFT_BIG_MAX];      // first chooser per candidate (1 KiB)
  uint8_t flags[SFT_BIG_MAX];  // 1 usable, 2 stereo
  int list[2 * (256 / SFT_BIG_WG + 1)];  // this workgroup's big nodes of a 256-node chunk: (node, KF2 node)
  int nlist;
  int wave_cnt[4];
};
static_assert(sizeof(SftBigLds) <= SFT_LDS_BYTES, "the big-node LDS aliases the wavefronts' 18 KiB");
struct SftMerge {  // one feature's passing bits and best key from its second wavefront
  uint64_t pm[SFT_BIG_MAX / 64];
  unsigned long long best;
};
static_assert(128 * sizeof(SftMerge) <= sizeof(float4) * SFT_BIG_MAX + sizeof(double) * SFT_BIG_MAX,
              "the merge slots of 128 features fit the candidates' xye + sig");

// index of node id `id` among fv2's ascending node ids, -1 if absent
__device__ __forceinline__ int sft_find_node(const orbfe_sft_pair& P, uint32_t id) {
  int lo = 0, hi = P.fv2.n_nodes - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t v = P.fv2.node_ids[mid];
    if (v == id) return mid;
    if (v < id) lo = mid + 1;
    else hi = mid - 1;
  }
  return -1;
}

__device__ void sft_big_nodes(const orbfe_sft_pair& P, int only_stereo, int b, SftBigLds& L) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const SftOctTab tab = sft_oct_tab(P);
  const float* F = P.f12;
  int base = 0;
  for (int a0 = 0; a0 < P.fv1.n_nodes; a0 += 256) {
  // 1. this workgroup's share of the chunk's big nodes, in node order
    if (t == 0) L.nlist = 0;
    const int a = a0 + t;
    int pairv = -1;
    if (a < P.fv1.n_nodes) {
      const int n1 = P.fv1.offsets[a + 1] - P.fv1.offsets[a];
      if (n1 > 0 && n1 <= SFT_BIG_MAX) {
        const int q = sft_find_node(P, P.fv1.node_ids[a]);
        if (q >= 0 && sft_big_node(n1, P.fv2.offsets[q + 1] - P.fv2.offsets[q])) pairv = q;
      }
    }
    const uint64_t m = wave_ballot(pairv >= 0);
    if (lane == 0) L.wave_cnt[w] = __popcll(m);
    __syncthreads();
    int rank = base + prefix_in_wave(m);
    for (int k = 0; k < w; k++) rank += L.wave_cnt[k];
    if (pairv >= 0 && rank % SFT_BIG_WG == b) {
      // this workgroup's ranks in the chunk are first, first + SFT_BIG_WG, ...: slots 0, 1, ...
      const int first = base + ((b - base % SFT_BIG_WG) + SFT_BIG_WG) % SFT_BIG_WG;
      const int slot = (rank - first) / SFT_BIG_WG;  // <= 256 / SFT_BIG_WG within the chunk
      L.list[2 * slot] = a;
      L.list[2 * slot + 1] = pairv;
      atomicMax(&L.nlist, slot + 1);
    }
    base += L.wave_cnt[0] + L.wave_cnt[1] + L.wave_cnt[2] + L.wave_cnt[3];
    __syncthreads();
    const int nlist = L.nlist;
  for (int e = 0; e < nlist; e++) {
    const int a = L.list[2 * e], q = L.list[2 * e + 1];
    const int o1 = P.fv1.offsets[a], n1 = P.fv1.offsets[a + 1] - o1;
    const int o2 = P.fv2.offsets[q], n2 = P.fv2.offsets[q + 1] - o2;
    // 2. candidates to LDS
    {
      SftCand c;
      sft_load_cand(P, o2, n2, t, only_stereo, tab, c);
      if (t < n2) {
        L.desc[t][0] = c.d0;
        L.desc[t][1] = c.d1;
        L.xye[t] = make_float4(c.x, c.y, c.epi_thr, 0.f);
        L.sig[t] = c.sig_thr;
        L.flags[t] = (c.usable ? 1 : 0) | (c.stereo ? 2 : 0);
      }
    }
    // 3. KF1 feature i of this thread: features in 64-lane chunks; with n1 <= 128 two wavefronts
    //    share a chunk (g = 0 / 1), each walking every other candidate, so all four wavefronts work
    const int G = n1 <= 128 ? 2 : 1, nchunk = 4 / G;
    const int chunk = w % nchunk, g = w / nchunk, i = 64 * chunk + lane;
    int idx1 = -1;
    bool ok1 = false, st1 = false;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    float la = 0.f, lb = 0.f, lc = 0.f, den = 0.f;
    if (i < n1) {
      idx1 = P.fv1.indices[o1 + i];
      st1 = P.kf1.u_right[idx1] >= 0;
      ok1 = P.kf1.mp_state[idx1] == ORBFE_MP_NONE && !(only_stereo && !st1);
      const orbfe_keypoint kp = P.kf1.keys_un[idx1];
      load_desc(P.kf1.descriptors + (size_t)idx1 * 32, a0, a1);
      la = kp.x * F[0] + kp.y * F[3] + F[6];  // CheckDistEpipolarLine :149-151
      lb = kp.x * F[1] + kp.y * F[4] + F[7];
      lc = kp.x * F[2] + kp.y * F[5] + F[8];
      den = la * la + lb * lb;
    }
    __syncthreads();
    // 4. passing set and round-0 choice: one pass over this thread's candidates p = g, g + G, ...
    //    (uniform LDS reads)
    uint64_t pm[SFT_BIG_MAX / 64] = {0, 0, 0, 0};
    unsigned long long best = ~0ull;
    if (ok1 && den != 0) {
      for (int p = g; p < n2; p += G) {
        if (!(L.flags[p] & 1)) continue;
        const int dist = hamming256(a0, a1, L.desc[p][0], L.desc[p][1]);
        if (dist > TH_LOW) continue;
        const float4 c = L.xye[p];
        if (!st1 && !(L.flags[p] & 2)) {
          const float dex = P.ex - c.x, dey = P.ey - c.y;
          if (dex * dex + dey * dey < c.z) continue;
        }
        const float num = la * c.x + lb * c.y + lc;
        const float dsqr = num * num / den;
        if (!((double)dsqr < L.sig[p])) continue;
        pm[p >> 6] |= 1ull << (p & 63);
        const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned long long)(0x7fffffff - p);
        best = key < best ? key : best;
      }
    }
    if (G == 2) {  // the g = 1 half's passing bits and best key join the g = 0 thread of the feature
      __syncthreads();  // (the merge slots alias the candidates' xye / sig, read until here)
      SftMerge* mg = reinterpret_cast<SftMerge*>(&L.xye[0]);
      if (g == 1) mg[i] = SftMerge{{pm[0], pm[1], pm[2], pm[3]}, best};
      __syncthreads();
      if (g == 0) {
        const SftMerge o = mg[i];
#pragma unroll
        for (int h = 0; h < SFT_BIG_MAX / 64; h++) pm[h] |= o.pm[h];
        best = o.best < best ? o.best : best;
      }
    }
    const bool owner = g == 0 && i < n1;  // the thread that carries feature i from here on
    int ch = !owner || best == ~0ull ? -1 : 0x7fffffff - (int)(best & 0xffffffffull);
    // 5. the claim order as a fixpoint over the node's features (feature i final after i rounds)
    for (int round = 0; round <= n1; round++) {
      if (t < n2) L.claim[t] = 0x7fffffff;
      __syncthreads();
      if (ch >= 0) atomicMin(&L.claim[ch], i);
      __syncthreads();
      unsigned long long bk = ~0ull;
      if (owner) {
#pragma unroll
        for (int h = 0; h < SFT_BIG_MAX / 64; h++) {
          uint64_t m = pm[h];
          while (m) {
            const int p = 64 * h + __builtin_ctzll(m);
            m &= m - 1;
            if (L.claim[p] < i) continue;  // vbMatched2: taken by an earlier feature of the node
            const unsigned long long key =
                ((unsigned long long)hamming256(a0, a1, L.desc[p][0], L.desc[p][1]) << 32) |
                (unsigned long long)(0x7fffffff - p);
            bk = key < bk ? key : bk;
          }
        }
      }
      const int nk = bk == ~0ull ? -1 : 0x7fffffff - (int)(bk & 0xffffffffull);
      const bool changed = nk != ch;
      ch = nk;
      if (!__syncthreads_or(changed)) break;
    }
    // 6. every feature of the node gets its final value (-1: no match)
    if (owner) P.match12[idx1] = ch >= 0 ? P.fv2.indices[o2 + ch] : -1;
    __syncthreads();  // the next node's candidates overwrite this one's
  }
  }
}

__global__ __launch_bounds__(256, 4) void k_sft_nodes(const orbfe_sft_pair* pairs, int only_stereo) {
  // per wave: the fixpoint path's node candidates, or the large-node path's claim bits beyond the
  // register chunks (a wave takes one path); a big-node workgroup's staging (SftBigLds) aliases
  // the same 18 KiB
  static_assert(SFT_MAX_NODE / 32 <= SFT_FP_MAX * 8, "claim bits fit the candidate area");
  __shared__ uint4 s_lds[SFT_LDS_BYTES / 16];
  uint32_t (*s_fp_desc)[SFT_FP_MAX * 8] = reinterpret_cast<uint32_t (*)[SFT_FP_MAX * 8]>(s_lds);
  int (*s_fp_claim)[SFT_FP_MAX] = reinterpret_cast<int (*)[SFT_FP_MAX]>(
      reinterpret_cast<uint8_t*>(s_lds) + 4 * SFT_FP_MAX * 8 * 4);
  // XCD-aware order: the workgroups of one pair run on one XCD, so its KeyFrames' keypoints,
  // descriptors and FeatureVectors are fetched into one L2 rather than eight
  const int2 blk = xcd_block2d();
  orbfe_sft_pair P = pairs[blk.y];
  sft_resolve_sizes(P);
  const int node_wgs = (int)gridDim.x - 1 - SFT_BIG_WG;
  if (blk.x > node_wgs) {  // the big-node workgroups of the pair
    if (P.kf2.n > SFT_MAX_KF2) return;
    sft_big_nodes(P, only_stereo, blk.x - node_wgs - 1, *reinterpret_cast<SftBigLds*>(s_lds));
    return;
  }
  if (blk.x == node_wgs) {
    // the last workgroup of a pair: KF1 features that no FeatureVector node lists -- a stopped
    // word (weight 0) is not added (TemplatedVocabulary.h:1198-1201) -- never match: -1. Disjoint
    // from the features the node wavefronts write, so no ordering is needed between them.
    uint32_t* bits = &s_fp_desc[0][0];  // 16 KiB = 131072 feature bits per round
    const int t = threadIdx.x;
    const int nidx = P.fv1.n_nodes > 0 ? P.fv1.offsets[P.fv1.n_nodes] : 0;
    for (int c0 = 0; c0 < P.kf1.n; c0 += 131072) {
      for (int i = t; i < 4096; i += 256) bits[i] = 0u;
      __syncthreads();
      for (int i = t; i < nidx; i += 256) {
        const int f = P.fv1.indices[i] - c0;
        if (f >= 0 && f < 131072) atomicOr(&bits[f >> 5], 1u << (f & 31));
      }
      __syncthreads();
      for (int f = c0 + t; f < min(P.kf1.n, c0 + 131072); f += 256)
        if (!((bits[(f - c0) >> 5] >> ((f - c0) & 31)) & 1u)) P.match12[f] = -1;
      __syncthreads();
    }
    return;
  }
  const int w = wave_id(), lane = lane_id();
  const int a = blk.x * 4 + w;
  if (a >= P.fv1.n_nodes) return;
  if (P.kf2.n > SFT_MAX_KF2) {  // over capacity (k_sft_finish reports ERR_CAPACITY): no matches
    for (int i = P.fv1.offsets[a] + lane_id(); i < P.fv1.offsets[a + 1]; i += 64) P.match12[P.fv1.indices[i]] = -1;
    return;
  }
  const uint32_t id = P.fv1.node_ids[a];
  const int o1 = P.fv1.offsets[a], e1 = P.fv1.offsets[a + 1];
  // the merge-join visits exactly the common node ids (:705-804): find id among KF2's node ids
  // with 64 independent loads per step (one round trip for the usual <= 64 .. 128 nodes)
  int lo = -1;
  for (int b = 0; b < P.fv2.n_nodes && lo < 0; b += 128) {
    const int i0 = b + lane, i1 = b + 64 + lane;
    const uint32_t v0 = i0 < P.fv2.n_nodes ? P.fv2.node_ids[i0] : ~0u;
    const uint32_t v1 = i1 < P.fv2.n_nodes ? P.fv2.node_ids[i1] : ~0u;
    const uint64_t m0 = wave_ballot(v0 == id), m1 = wave_ballot(v1 == id);
    if (m0) lo = b + __builtin_ctzll(m0);
    else if (m1) lo = b + 64 + __builtin_ctzll(m1);
  }
  if (lo < 0) {  // no common node (the merge-join skips it): no matches for these features
    for (int i = o1 + lane; i < e1; i += 64) P.match12[P.fv1.indices[i]] = -1;
    return;
  }
  const int o2 = P.fv2.offsets[lo], n2 = P.fv2.offsets[lo + 1] - o2;
  if (sft_big_node(e1 - o1, n2)) return;  // a big-node workgroup of the pair writes this node
  if (e1 - o1 <= 64 && n2 <= 64) {
    sft_node_fixpoint<1>(P, o1, e1 - o1, o2, n2, only_stereo, s_fp_desc[w], s_fp_claim[w]);
    return;
  }
  // large nodes: -1 first, stored before the walk's matches overwrite some of them (the wait
  // orders the two stores to one address from different lanes)
  for (int i = o1 + lane; i < e1; i += 64) P.match12[P.fv1.indices[i]] = -1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t* far = s_fp_desc[w];
  if (n2 > SFT_REG_CHUNKS * 64)
    for (int i = lane; i < (n2 + 31) / 32; i += 64) far[i] = 0;
  const SftOctTab tab = sft_oct_tab(P);
  SftCand c0, c1, c2, c3;
  sft_load_cand(P, o2, n2, lane, only_stereo, tab, c0);
  sft_load_cand(P, o2, n2, 64 + lane, only_stereo, tab, c1);
  sft_load_cand(P, o2, n2, 128 + lane, only_stereo, tab, c2);
  sft_load_cand(P, o2, n2, 192 + lane, only_stereo, tab, c3);
  bool cl0 = false, cl1 = false, cl2 = false, cl3 = false;
  const float* F = P.f12;
  const float f0 = F[0], f1 = F[1], f2 = F[2], f3 = F[3], f4 = F[4], f5 = F[5], f6 = F[6],
              f7 = F[7], f8 = F[8];
  // KF1 features of the node, 64 at a time: each lane preloads one (index, usable, position,
  // descriptor); the sequential walk below broadcasts them with readlane (no global round trip
  // per step of the claim order)
  for (int b1 = o1; b1 < e1; b1 += 64) {
    const int my = b1 + lane;
    int m_idx = -1;
    bool m_ok = false, m_st = false;
    float m_x = 0.f, m_y = 0.f;
    uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
    if (my < e1) {
      m_idx = P.fv1.indices[my];
      m_st = P.kf1.u_right[m_idx] >= 0;
      m_ok = P.kf1.mp_state[m_idx] == ORBFE_MP_NONE && !(only_stereo && !m_st);
      const orbfe_keypoint k1 = P.kf1.keys_un[m_idx];
      m_x = k1.x;
      m_y = k1.y;
      load_desc(P.kf1.descriptors + (size_t)m_idx * 32, m0, m1);
    }
    const uint64_t okmask = wave_ballot(m_ok);
    const int nb = min(64, e1 - b1);
  for (int q = 0; q < nb; q++) {
    if (!((okmask >> q) & 1ull)) continue;  // has a MapPoint, or mono under bOnlyStereo
    const int idx1 = __builtin_amdgcn_readlane(m_idx, q);
    const bool st1 = __builtin_amdgcn_readlane((int)m_st, q) != 0;
    orbfe_keypoint kp1;
    kp1.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m_x), q));
    kp1.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m_y), q));
    uint4 a0, a1;
    a0.x = __builtin_amdgcn_readlane(m0.x, q);
    a0.y = __builtin_amdgcn_readlane(m0.y, q);
    a0.z = __builtin_amdgcn_readlane(m0.z, q);
    a0.w = __builtin_amdgcn_readlane(m0.w, q);
    a1.x = __builtin_amdgcn_readlane(m1.x, q);
    a1.y = __builtin_amdgcn_readlane(m1.y, q);
    a1.z = __builtin_amdgcn_readlane(m1.z, q);
    a1.w = __builtin_amdgcn_readlane(m1.w, q);
    // epipolar line l = x1' F12 (CheckDistEpipolarLine :149-151)
    const float la = kp1.x * f0 + kp1.y * f3 + f6;
    const float lb = kp1.x * f1 + kp1.y * f4 + f7;
    const float lc = kp1.x * f2 + kp1.y * f5 + f8;
    const float den = la * la + lb * lb;
    unsigned long long best = sft_key(c0, cl0, lane, a0, a1, st1, P.ex, P.ey, la, lb, lc, den);
    unsigned long long k;
    if (n2 > 64) {
      k = sft_key(c1, cl1, 64 + lane, a0, a1, st1, P.ex, P.ey, la, lb, lc, den);
      best = k < best ? k : best;
    }
    if (n2 > 128) {
      k = sft_key(c2, cl2, 128 + lane, a0, a1, st1, P.ex, P.ey, la, lb, lc, den);
      best = k < best ? k : best;
    }
    if (n2 > 192) {
      k = sft_key(c3, cl3, 192 + lane, a0, a1, st1, P.ex, P.ey, la, lb, lc, den);
      best = k < best ? k : best;
    }
    for (int cbase = SFT_REG_CHUNKS * 64; cbase < n2; cbase += 64) {  // very large nodes
      SftCand cx;
      const int p = cbase + lane;
      sft_load_cand(P, o2, n2, p, only_stereo, tab, cx);
      const bool clx = p < n2 && ((far[p >> 5] >> (p & 31)) & 1u);
      k = sft_key(cx, clx, p, a0, a1, st1, P.ex, P.ey, la, lb, lc, den);
      best = k < best ? k : best;
    }
    best = wave_min_u64(best);
    if (best != ~0ull) {
      const int p = 0x7fffffff - (int)(best & 0xffffffffull);
      // vbMatched2[bestIdx2] = true (:776): the owning lane marks its candidate claimed
      cl0 = cl0 || (p == lane);
      cl1 = cl1 || (p == 64 + lane);
      cl2 = cl2 || (p == 128 + lane);
      cl3 = cl3 || (p == 192 + lane);
      if (lane == 0) {
        P.match12[idx1] = P.fv2.indices[o2 + p];
        if (p >= SFT_REG_CHUNKS * 64) far[p >> 5] |= 1u << (p & 31);
      }
      if (p >= SFT_REG_CHUNKS * 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
    }
  }
  }
}

__global__ __launch_bounds__(256) void k_sft_finish(const orbfe_sft_pair* pairs, int check_ori) {
  __shared__ int s_hist[HISTO_LENGTH];
  __shared__ int s_misc[8];
  orbfe_sft_pair P = pairs[blockIdx.x];
  sft_resolve_sizes(P);
  const int t = threadIdx.x, lane = lane_id();
  if (t < HISTO_LENGTH) s_hist[t] = 0;
  if (t == 0) s_misc[4] = 0;
  __syncthreads();
  if (P.kf2.n > SFT_MAX_KF2) {
    if (t == 0) *P.nmatches = ORBFE_ERR_CAPACITY;
    return;
  }
  if (check_ori) {  // rotation consistency (:806-826)
    for (int i = t; i < P.kf1.n; i += 256) {
      const int m = P.match12[i];
      if (m >= 0) atomicAdd(&s_hist[rot_bin_dev(P.kf1.keys_un[i].angle, P.kf2.keys_un[m].angle)], 1);
    }
    __syncthreads();
    if (t == 0) three_maxima_dev(s_hist, s_misc[0], s_misc[1], s_misc[2]);
    __syncthreads();
    const int i1 = s_misc[0], i2 = s_misc[1], i3 = s_misc[2];
    for (int i = t; i < P.kf1.n; i += 256) {
      const int m = P.match12[i];
      if (m >= 0) {
        const int bin = rot_bin_dev(P.kf1.keys_un[i].angle, P.kf2.keys_un[m].angle);
        if (bin != i1 && bin != i2 && bin != i3) P.match12[i] = -1;
      }
    }
    __syncthreads();
  }
  int cnt = 0;
  for (int i = t; i < P.kf1.n; i += 256) cnt += P.match12[i] >= 0;
  cnt = wave_sum(cnt);
  if (lane == 0) atomicAdd(&s_misc[4], cnt);
  __syncthreads();
  if (t == 0) *P.nmatches = s_misc[4];
}

// ---------------------------------------------------------------------------------------------
// Frame grid (AssignFeaturesToGrid) as CSR: start[GRID_CELLS + 1], items[n]
struct GridArgs {
  const orbfe_keypoint* keys;
  const float* u_right;
  int n;
  float min_x, min_y, inv_w, inv_h;
  int32_t* start;
  uint4* recs;  // per grid item: {x, y, uRight (float bits), index | octave << 16}
};

// Counting sort by cell (1024 threads): cell histogram, scan, scatter, then each cell's few
// items put back in ascending keypoint order (mGrid[i][j] is filled in index order, Frame.cc:286-293,
// and GetFeaturesInArea's candidate order decides ties).
__global__ __launch_bounds__(1024) void k_grid(GridArgs g) {
  extern __shared__ int s_grid[];  // GRID_CELLS + 1 counters, 16 scan ints, then n items
  int* cnt = s_grid;
  int* wsum = s_grid + GRID_CELLS + 1;
  int* items = wsum + 16;
  const int t = threadIdx.x;
  auto cell_of = [&](int i) {
    const orbfe_keypoint kp = g.keys[i];
    // PosInGrid (Frame.cc:435-445): round() half away from zero on the float product
    const int px = (int)roundf((kp.x - g.min_x) * g.inv_w);
    const int py = (int)roundf((kp.y - g.min_y) * g.inv_h);
    return (px >= 0 && px < GRID_COLS && py >= 0 && py < GRID_ROWS) ? px * GRID_ROWS + py : -1;
  };
  for (int c = t; c <= GRID_CELLS; c += 1024) cnt[c] = 0;
  __syncthreads();
  for (int i = t; i < g.n; i += 1024) {
    const int c = cell_of(i);
    if (c >= 0) atomicAdd(&cnt[c], 1);
  }
  __syncthreads();
  block_scan_excl_1024(cnt, GRID_CELLS + 1, wsum);
  for (int c = t; c <= GRID_CELLS; c += 1024) g.start[c] = cnt[c];  // start[GRID_CELLS] = keys in grid
  __syncthreads();
  for (int i = t; i < g.n; i += 1024) {
    const int c = cell_of(i);
    if (c >= 0) items[atomicAdd(&cnt[c], 1)] = i;
  }
  __syncthreads();
  // cnt[c] is now the end of cell c; its start is the end of cell c - 1
  for (int c = t; c < GRID_CELLS; c += 1024) {
    const int b = c ? cnt[c - 1] : 0, e = cnt[c];
    for (int x = b + 1; x < e; x++) {  // insertion sort of the cell's items (a handful)
      const int v = items[x];
      int y = x - 1;
      while (y >= b && items[y] > v) {
        items[y + 1] = items[y];
        y--;
      }
      items[y + 1] = v;
    }
  }
  __syncthreads();
  const int total = cnt[GRID_CELLS - 1];
  for (int i = t; i < total; i += 1024) {  // the fields the window walks read, in one 16-B record
    const int k = items[i];
    const orbfe_keypoint kp = g.keys[k];
    g.recs[i] = make_uint4(__float_as_uint(kp.x), __float_as_uint(kp.y), __float_as_uint(g.u_right[k]),
                           (unsigned)k | ((unsigned)kp.octave << 16));
  }
}

// ---------------------------------------------------------------------------------------------
// SearchByProjection (both overloads): queries + fixpoint rounds + finish

struct SbpArgs {
  orbfe_frame_view F;        // device pointers
  const int32_t* grid_start;
  const uint4* grid_recs;
  const SbpQuery* q;
  const uint8_t* qdesc;       // m x 32
  int m;
  int mode;                   // 0 local (best + second + ratio), 1 first minimum (other overloads)
  float nnratio;
  int dist_th;                // accept bestDist <= dist_th (TH_HIGH, TH_LOW or ORBdist)
  int block_any;              // pre-blocked keypoints: SBP_BLOCK_*
  int cand_cap;               // per-query candidate cache entries
  int no_claims;              // no query blocks a keypoint: round 0 is the result
  int32_t* res_prev;
  int32_t* res_cur;
  const int32_t* owner_prev;  // INT_MAX = unclaimed in the previous round
  int32_t* owner_cur;
  int32_t* owner_next;        // cleared by this round for the next one
  int32_t* state;             // [0] converged flag, [1] rounds run, [2 + r] changed in round r
  int round;
  // per-query candidate cache filled in round 0 (keypoints passing the window, level and stereo
  // gates, in GetFeaturesInArea order, with their distances; one dword each, cand_pack); later
  // rounds only re-apply the claims. cand_n[i] < 0: more than cand_cap candidates, the query
  // re-searches every round. Candidates at distance 256 are left out: they can be neither best
  // nor second (:106-118).
  uint32_t* cand;
  int32_t* cand_n;
  // rounds >= 2 with the cache: round r-2's owners (round r compares them with round r-1's and
  // re-evaluates only the queries a changed keypoint can reach); NULL: every query is re-evaluated
  const int32_t* owner_rm2;
  // round 0 before k_sbp_sweep: a query none of whose candidates (pre-blocked ones aside) is within
  // dist_th can never match, whatever the claims -- blocking only removes candidates -- so it
  // leaves the claim order: cand_n = 0 (its round-0 result, -1, is final)
  int prune;
  uint32_t* live;  // with prune: bit i set for every query left in the claim order (k_sbp_sweep)
  // round 0: candidates at a distance >= keep_below are not cached (256: all are). Such a
  // candidate can never decide a result (sbp_keep_below), so the claim order runs on the rest.
  int keep_below;
};

// A keypoint whose owner changed from o1 to o2 between rounds: blocked(k) = owner < q flips exactly
// for the queries lo < q <= hi (lo = min, hi = max of the two owners), and only a query whose
// window (|x - kx| < r and |y - ky| < r, the test every candidate passed) holds the keypoint can
// have it as a candidate. A query no entry reaches keeps its previous result.
struct SbpChange {
  float x, y;
  int lo, hi;
};
#define SBP_CHG_MAX 256  // more changed keypoints than this: the round re-evaluates every query

// Keypoint taken before the search starts: Frame::mvpMapPoints with Observations() > 0 (:91-93,
// :1420-1422) or any non-NULL entry (:384, :1567).
__device__ __forceinline__ bool sbp_pre_blocked(const SbpArgs& a, int k) {
  if (a.block_any == SBP_BLOCK_NONE) return false;  // Fuse, SearchBySim3: nothing is skipped
  const uint8_t st = a.F.mp_state[k];
  return a.block_any == SBP_BLOCK_ANY ? st != ORBFE_MP_NONE : st == ORBFE_MP_OBSERVED;
}

// Window candidate test that precedes the distance (rec = {x, y, uRight, index | octave << 16}).
__device__ __forceinline__ bool sbp_gate(const SbpQuery& q, const uint4& rec, const float* level_sigma2) {
  const float ur = __uint_as_float(rec.z);
  if (q.gate == SBP_GATE_STEREO) return !(ur > 0 && fabsf(q.xr - ur) > q.er_lim);
  if (q.gate == SBP_GATE_FUSE) {  // Fuse (:930-954): reprojection error against chi2 bounds
    const float inv = 1.0f / level_sigma2[rec.w >> 16];  // mvInvLevelSigma2 (ORBextractor.cc:433)
    const float ex = q.x - __uint_as_float(rec.x), ey = q.y - __uint_as_float(rec.y);
    if (ur >= 0) {
      const float er = q.xr - ur;
      const float e2 = ex * ex + ey * ey + er * er;
      return !((double)(e2 * inv) > 7.8);
    }
    const float e2 = ex * ex + ey * ey;
    return !((double)(e2 * inv) > 5.99);
  }
  return true;
}

// One MapPoint's search given a predicate blocked(k). Returns the keypoint index or -1.
// Best / second-best bookkeeping of the reference loop (:106-118 local; :1417-1450 last frame).
struct SbpBest {
  int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
  __device__ __forceinline__ void add(int mode, int dist, int level, int k) {
    if (mode == 0) {
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = level;
        bestIdx = k;
      } else if (dist < bestDist2) {
        bestLevel2 = level;
        bestDist2 = dist;
      }
    } else if (dist < bestDist) {
      bestDist = dist;
      bestIdx = k;
    }
  }
  __device__ __forceinline__ int result(int mode, float nnratio, int dist_th) const {
    if (bestDist > dist_th) return -1;
    if (mode == 0 && bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) return -1;
    return bestIdx;
  }
};

// Round > 0 with a cached candidate list: only the claims changed.
template <class Blocked>
__device__ int sbp_cached(const SbpArgs& a, int i, int n, Blocked blocked) {
  SbpBest b;
  const uint32_t* ce = a.cand + (size_t)i * a.cand_cap;
  for (int c = 0; c < n; c++) {
    const uint32_t e = ce[c];
    const int k = cand_key(e);
    if (blocked(k)) continue;
    b.add(a.mode, cand_dist(e), cand_level(e), k);
  }
  return b.result(a.mode, a.nnratio, a.dist_th);
}

template <class Blocked, bool RECORD = false>
__device__ int sbp_one(const SbpArgs& a, int i, Blocked blocked) {
  const SbpQuery q = a.q[i];
  if (RECORD) a.cand_n[i] = 0;
  if (!(q.flags & 1)) return -1;
  const orbfe_frame_view& F = a.F;
  const float x = q.x, y = q.y, r = q.r;
  // GetFeaturesInArea (Frame.cc:376-433)
  const int nMinCellX = max(0, (int)floorf((x - F.min_x - r) * F.grid_inv_w));
  if (nMinCellX >= GRID_COLS) return -1;
  const int nMaxCellX = min(GRID_COLS - 1, (int)ceilf((x - F.min_x + r) * F.grid_inv_w));
  if (nMaxCellX < 0) return -1;
  const int nMinCellY = max(0, (int)floorf((y - F.min_y - r) * F.grid_inv_h));
  if (nMinCellY >= GRID_ROWS) return -1;
  const int nMaxCellY = min(GRID_ROWS - 1, (int)ceilf((y - F.min_y + r) * F.grid_inv_h));
  if (nMaxCellY < 0) return -1;
  const bool checkLevels = (q.min_level > 0) || (q.max_level >= 0);
  uint4 dq0, dq1;
  load_desc(a.qdesc + (size_t)i * 32, dq0, dq1);
  SbpBest b;
  int nc = 0;
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      const int c = ix * GRID_ROWS + iy;
      const int e = a.grid_start[c + 1];
      for (int j = a.grid_start[c]; j < e; j++) {
        const uint4 rec = a.grid_recs[j];
        const int k = (int)(rec.w & 0xffffu);
        struct {
          float x, y;
          int octave;
        } kp = {__uint_as_float(rec.x), __uint_as_float(rec.y), (int)(rec.w >> 16)};
        if (checkLevels) {
          if (kp.octave < q.min_level) continue;
          if (q.max_level >= 0 && kp.octave > q.max_level) continue;
        }
        const float distx = kp.x - x, disty = kp.y - y;
        if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
        if (!RECORD && blocked(k)) continue;
        if (!sbp_gate(q, rec, F.level_sigma2)) continue;
        uint4 d0, d1;
        load_desc(F.descriptors + (size_t)k * 32, d0, d1);
        const int dist = hamming256(dq0, dq1, d0, d1);
        if (RECORD) {
          if (dist == 256) continue;
          if (nc < a.cand_cap) a.cand[(size_t)i * a.cand_cap + nc] = cand_pack(k, dist, kp.octave);
          nc++;
          if (blocked(k)) continue;
        }
        b.add(a.mode, dist, kp.octave, k);
      }
    }
  }
  if (RECORD) a.cand_n[i] = nc <= a.cand_cap ? nc : -1;
  return b.result(a.mode, a.nnratio, a.dist_th);
}

struct SbpInit {
  int32_t *res0, *res1, *own0, *own2, *state, *nmatches, *serial;
  uint32_t* live;  // the sweep's live-query bitmap (NULL: none)
  int nq, nf;
};
// One launch for the per-call initialisation (results "never", owners unclaimed, counters 0).
__global__ __launch_bounds__(256) void k_sbp_init(SbpInit in) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < in.nq) {
    in.res0[i] = (int32_t)0xfefefefe;  // never a result
    in.res1[i] = (int32_t)0xfefefefe;
  }
  if (in.live && i < (in.nq + 31) / 32) in.live[i] = 0u;
  if (i < in.nf) {
    in.own0[i] = 0x7fffffff;
    in.own2[i] = 0x7fffffff;
  }
  if (i < SBP_ROUND_CAP + 4) in.state[i] = 0;
  if (i < 16) in.serial[i] = 0;  // [0] serial walk, [1..9] k_sbp_sweep's statistics
  if (i == 0) *in.nmatches = 0;
}

__global__ __launch_bounds__(256) void k_sbp_round(SbpArgs a) {
  __shared__ SbpChange s_chg[SBP_CHG_MAX];
  __shared__ int s_nchg;
  if (a.round > 1 && a.state[2 + a.round - 1] == 0) {  // previous round reproduced its input
    if (blockIdx.x == 0 && threadIdx.x == 0) a.state[0] = 1;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.state[1] = a.round + 1;
  // the keypoints whose owner differs between rounds r-2 and r-1, gathered by every workgroup
  // (owner_rm2 is not written during this round: four owner buffers rotate)
  int nchg = SBP_CHG_MAX + 1;
  if (a.owner_rm2) {
    if (threadIdx.x == 0) s_nchg = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < a.F.n; k += 256) {
      const int o1 = a.owner_rm2[k], o2 = a.owner_prev[k];
      if (o1 != o2) {
        const int slot = atomicAdd(&s_nchg, 1);
        if (slot < SBP_CHG_MAX) {
          SbpChange c;
          c.x = a.F.keys_un[k].x;
          c.y = a.F.keys_un[k].y;
          c.lo = min(o1, o2);
          c.hi = max(o1, o2);
          s_chg[slot] = c;
        }
      }
    }
    __syncthreads();
    nchg = s_nchg;
  }
  const bool sparse = nchg <= SBP_CHG_MAX;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.F.n) a.owner_next[i] = 0x7fffffff;
  bool changed = false;
  if (i < a.m) {
    bool need = true;
    if (sparse) {
      const float qx = a.q[i].x, qy = a.q[i].y, qr = a.q[i].r;
      need = false;
      for (int c = 0; c < nchg && !need; c++) {
        const SbpChange e = s_chg[c];
        need = e.lo < i && i <= e.hi && fabsf(e.x - qx) < qr && fabsf(e.y - qy) < qr;
      }
    }
    auto blocked = [&](int k) { return sbp_pre_blocked(a, k) || a.owner_prev[k] < i; };
    int res;
    if (!need) {
      res = a.res_prev[i];  // no candidate changed its blocked state for this query
    } else if (!a.cand_n) {
      res = sbp_one(a, i, blocked);
    } else if (a.round == 0) {
      res = sbp_one<decltype(blocked), true>(a, i, blocked);
    } else {
      const int n = a.cand_n[i];
      res = n >= 0 ? sbp_cached(a, i, n, blocked) : sbp_one(a, i, blocked);
    }
    a.res_cur[i] = res;
    if (res >= 0 && (a.q[i].flags & 2)) atomicMin(&a.owner_cur[res], i);
    changed = res != a.res_prev[i];
  }
  // "some result changed": a plain store of 1 (every writer stores the same value). A device-scope
  // atomic on one address is serialised at the coherence point across the XCDs (~10 ns each):
  // one per query or per wavefront was most of this kernel's time.
  if (wave_ballot(changed) && lane_id() == 0) a.state[2 + a.round] = 1;
}

// Round 0 with the candidate cache, 16 lanes (one DPP row) per MapPoint. The window's grid cells
// are taken 16 at a time in GetFeaturesInArea order (ix outer, iy inner, Frame.cc:394-430), one
// cell per lane: a counting pass and a 16-lane scan place each lane's candidates in that order in
// the cache, then a second pass computes their distances. The sequential best / second-best
// bookkeeping of :106-118 / :1417-1450 equals the two smallest (dist, position) keys over the
// unblocked candidates with dist < 256, so each lane keeps its two smallest and the row merges.
__device__ __forceinline__ unsigned long long min_u64(unsigned long long a, unsigned long long b) {
  return a < b ? a : b;
}
__device__ __forceinline__ unsigned long long max_u64(unsigned long long a, unsigned long long b) {
  return a < b ? b : a;
}
#define SBP_FLAT 128  // flattened grid items per 16-lane row and pass (LDS)
__global__ __launch_bounds__(256) void k_sbp_round0(SbpArgs a) {
  __shared__ int s_flat[16][SBP_FLAT];
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.state[1] = 1;
    if (a.no_claims) a.state[0] = 1;  // nothing to iterate: converged after this round
  }
  if (t < a.F.n) a.owner_next[t] = 0x7fffffff;
  const int j = threadIdx.x & 15, row = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + row;
  if (i >= a.m) return;  // the 16 lanes of a row leave together; rows sync with wave_sync only
  int* flat = s_flat[row];
  const SbpQuery q = a.q[i];
  const orbfe_frame_view& F = a.F;
  const float x = q.x, y = q.y, r = q.r;
  int nMinCellX = 0, nMaxCellX = -1, nMinCellY = 0, nMaxCellY = -1;
  if (q.flags & 1) {  // GetFeaturesInArea's cell range (Frame.cc:383-397); empty when out of grid
    nMinCellX = max(0, (int)floorf((x - F.min_x - r) * F.grid_inv_w));
    nMaxCellX = min(GRID_COLS - 1, (int)ceilf((x - F.min_x + r) * F.grid_inv_w));
    nMinCellY = max(0, (int)floorf((y - F.min_y - r) * F.grid_inv_h));
    nMaxCellY = min(GRID_ROWS - 1, (int)ceilf((y - F.min_y + r) * F.grid_inv_h));
    if (nMinCellX >= GRID_COLS || nMaxCellX < 0 || nMinCellY >= GRID_ROWS || nMaxCellY < 0)
      nMaxCellX = nMinCellX - 1;
  }
  const int ny = nMaxCellY - nMinCellY + 1;
  const int ncell = nMaxCellX >= nMinCellX && ny > 0 ? (nMaxCellX - nMinCellX + 1) * ny : 0;
  const bool checkLevels = (q.min_level > 0) || (q.max_level >= 0);
  uint4 dq0 = make_uint4(0, 0, 0, 0), dq1 = dq0;
  if (ncell) load_desc(a.qdesc + (size_t)i * 32, dq0, dq1);
  uint32_t* ce = a.cand + (size_t)i * a.cand_cap;
  const unsigned long long NONE = ~0ull;
  unsigned long long k1 = NONE, k2 = NONE;  // (dist << 40 | position << 8 | level)
  int kb1 = -1;                             // keypoint of k1
  int total = 0;                            // candidates so far, in GetFeaturesInArea order
  const int rowbase = (threadIdx.x & 63) & ~15;  // first lane of this row in the wavefront
  for (int o0 = 0; o0 < ncell; o0 += 16) {
    // 16 cells, one per lane: item ranges and their offsets in the flattened list
    const int o = o0 + j;
    int b = 0, e = 0;
    if (o < ncell) {
      const int c = (nMinCellX + o / ny) * GRID_ROWS + nMinCellY + o % ny;
      b = a.grid_start[c];
      e = a.grid_start[c + 1];
    }
    const int cnt = e - b;
    int inc = cnt;
#pragma unroll
    for (int s2 = 1; s2 < 16; s2 <<= 1) {
      const int y2 = __shfl_up(inc, s2, 16);
      if (j >= s2) inc += y2;
    }
    const int nflat = __shfl(inc, 15, 16), off = inc - cnt;
    for (int f0 = 0; f0 < nflat; f0 += SBP_FLAT) {
      for (int u = max(off, f0); u < min(off + cnt, f0 + SBP_FLAT); u++) flat[u - f0] = b + (u - off);
      wave_sync();
      const int nf = min(nflat - f0, SBP_FLAT);
      for (int u0 = 0; u0 < nf; u0 += 16) {
        const int u = u0 + j;
        bool pass = false;
        int k = 0, oct = 0, dist = 256;
        if (u < nf) {  // window / level / stereo gates of :86-103, :1412-1427
          const uint4 rec = a.grid_recs[flat[u]];
          k = (int)(rec.w & 0xffffu);
          oct = (int)(rec.w >> 16);
          pass = true;
          if (checkLevels) {
            if (oct < q.min_level) pass = false;
            if (q.max_level >= 0 && oct > q.max_level) pass = false;
          }
          const float distx = __uint_as_float(rec.x) - x, disty = __uint_as_float(rec.y) - y;
          if (!(fabsf(distx) < r && fabsf(disty) < r)) pass = false;
          if (pass && !sbp_gate(q, rec, F.level_sigma2)) pass = false;
        }
        if (pass) {
          uint4 d0, d1;
          load_desc(F.descriptors + (size_t)k * 32, d0, d1);
          dist = hamming256(dq0, dq1, d0, d1);
        }
        const bool keep = pass && dist < a.keep_below;  // 256: never best or second (sbp_keep_below)
        const uint64_t bm = (wave_ballot(keep) >> rowbase) & 0xffffull;
        if (keep) {
          const int pos = total + __popcll(bm & ((1ull << j) - 1));
          if (pos < a.cand_cap) ce[pos] = cand_pack(k, dist, oct);
          if (!sbp_pre_blocked(a, k)) {  // blocked(k) in round 0
            const unsigned long long key =
                ((unsigned long long)dist << 40) | ((unsigned long long)pos << 8) | (unsigned)oct;
            if (key < k1) {
              k2 = k1;
              k1 = key;
              kb1 = k;
            } else if (key < k2) {
              k2 = key;
            }
          }
        }
        total += __popcll(bm);
      }
      wave_sync();  // the row's flat list is rewritten by the next pass
    }
  }
  // top-2 over the row (the keypoint of the smallest key travels with it)
#pragma unroll
  for (int s2 = 8; s2 > 0; s2 >>= 1) {
    const unsigned long long o1 = __shfl_xor(k1, s2, 16), o2 = __shfl_xor(k2, s2, 16);
    const int ob = __shfl_xor(kb1, s2, 16);
    k2 = min_u64(max_u64(k1, o1), min_u64(k2, o2));
    if (o1 < k1) {
      k1 = o1;
      kb1 = ob;
    }
  }
  if (j != 0) return;
  // pruned: the smallest unblocked distance exceeds dist_th, so no claim order can make a match
  const bool dead = a.prune && (k1 == NONE || (int)(k1 >> 40) > a.dist_th);
  a.cand_n[i] = dead ? 0 : total <= a.cand_cap ? total : -1;
  if (a.live && !dead) atomicOr(&a.live[i >> 5], 1u << (i & 31));
  int res = -1;
  if (k1 != NONE) {
    SbpBest bb;
    bb.bestDist = (int)(k1 >> 40);
    bb.bestLevel = (int)(k1 & 0xff);
    bb.bestIdx = kb1;
    if (k2 != NONE) {
      bb.bestDist2 = (int)(k2 >> 40);
      bb.bestLevel2 = (int)(k2 & 0xff);
    }
    res = bb.result(a.mode, a.nnratio, a.dist_th);
  }
  a.res_cur[i] = res;
  if (res >= 0 && (q.flags & 2)) atomicMin(&a.owner_cur[res], i);
  const uint64_t changed = wave_ballot(res != a.res_prev[i]);  // plain store, see k_sbp_round
  if (changed && lane_id() == __ffsll((long long)wave_ballot(true)) - 1) a.state[2] = 1;
}

// ---- the claim order after round 0: one workgroup, query chunk by query chunk ------------------
// The reference assigns in query order (:51-130 local, :1371-1450 last frame): query i skips a
// keypoint an earlier query took (mvpMapPoints[k] set, with Observations() > 0 for the local map),
// so result(i) depends on the results of the queries before it -- a chain the grid-wide rounds
// resolve one link per launch (8-23 rounds on the C5 scene, ~12 us each). Here round 0 (grid-wide)
// fills the candidate cache with the candidates that can decide a result (sbp_keep_below) and
// prunes the queries that can never match (no candidate within dist_th outside the pre-blocked
// keypoints: cand_n = 0, no bit in the live bitmap), and one 1024-thread workgroup walks the live
// queries in ascending order, a chunk of up to 1024 at a time:
//   * a window of the live bitmap (SWEEP_WINDOW_WORDS words) is compacted into an LDS list, order
//     kept; full chunks of the list are processed, the remainder carried over;
//   * a chunk's cache entries are staged in an LDS pool (a block scan of the counts; a chunk ends
//     where the pool is full);
//   * within the chunk, Jacobi rounds on LDS state: every query re-evaluates from its pooled entries
//     with blocked(k) = taken[k] (pre-blocked or claimed by an earlier chunk -- every such query
//     index is smaller) or own[k] < i (own[k] = the smallest chunk query whose current result is k
//     and whose assignment blocks it), until a round reproduces the previous one. The sequential
//     results are the unique fixpoint of that map (result(i) depends only on earlier queries), and
//     after r rounds the chunk's first r queries hold them, so a chunk of C queries settles within
//     C + 1 rounds; chains inside one chunk are short (a few rounds); the chunk's claims are then
//     committed to taken[];
//   * a chunk still moving after max_rounds rounds (a debug knob: orbfe_debug_matcher_set_sweep)
//     falls back to the reference loop over that chunk, one thread in query order.
// Results of the live queries are written over round 0's (which are final for the pruned ones).
struct SbpSweepArgs {
  int32_t* res;     // round 0's result buffer, the live queries' results written in place
  int chunk;        // live queries per chunk (1 .. SWEEP_THREADS)
  int max_rounds;   // Jacobi rounds per chunk before the sequential walk
  int32_t* stats;   // see orbfe_debug_matcher_sweep_stats
};

#define SWEEP_WINDOW_WORDS 512  // live-bitmap words compacted per window (16,384 queries)
#define SWEEP_LIST (SWEEP_WINDOW_WORDS * 32 + SWEEP_THREADS)
#define SWEEP_E 12              // cache entries a query keeps in registers for its chunk
__host__ __device__ inline size_t sweep_lds(int n) {
  // four owner arrays own[4][n] (three rotating, one base: -1 where a keypoint is taken), the live
  // list (a window plus a chunk's remainder)
  return sizeof(int) * (4 * (size_t)n + SWEEP_LIST);
}

// result of query i from its cache (or the grid walk past the cache) under `blocked`
template <class Blocked>
__device__ __forceinline__ int sbp_eval(const SbpArgs& a, int i, Blocked blocked) {
  const int n = a.cand_n[i];
  return n < 0 ? sbp_one(a, i, blocked) : sbp_cached(a, i, n, blocked);
}

// inclusive prefix sum over the workgroup (SWEEP_THREADS threads); *total = the sum
__device__ __forceinline__ int sweep_scan_incl(int v, int* wsum, int* total) {
  const int ln = lane_id(), wv = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (ln >= o) inc += y;
  }
  if (ln == 63) wsum[wv] = inc;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < SWEEP_THREADS / 64; q++) {
    const int x = wsum[q];
    if (q < wv) off += x;
    tot += x;
  }
  __syncthreads();  // wsum is free again
  *total = tot;
  return off + inc;
}

// The reference's best / second-best bookkeeping over cache entries in order (:106-118 / :1417-
// 1450) is the two smallest (distance, position) keys over the unblocked entries (see
// k_sbp_round0); as 32-bit keys distance << 17 | position << 5 | octave (position < 4096, octave <
// 32), kept branch-free by min / max.
__device__ __forceinline__ uint32_t sweep_key(uint32_t e, int pos) {
  return ((uint32_t)cand_dist(e) << 17) | ((uint32_t)pos << 5) | (uint32_t)cand_level(e);
}
__device__ __forceinline__ int sweep_result(const SbpArgs& a, uint32_t k1, uint32_t k2, int k1_key) {
  if (k1 == 0xffffffffu) return -1;
  SbpBest b;
  b.bestDist = (int)(k1 >> 17);
  b.bestLevel = (int)(k1 & 31u);
  b.bestIdx = k1_key;
  if (k2 != 0xffffffffu) {
    b.bestDist2 = (int)(k2 >> 17);
    b.bestLevel2 = (int)(k2 & 31u);
  }
  return b.result(a.mode, a.nnratio, a.dist_th);
}

__global__ __launch_bounds__(SWEEP_THREADS) void k_sbp_sweep(SbpArgs a, SbpSweepArgs s) {
  extern __shared__ int s_lds[];
  __shared__ int s_wsum[SWEEP_THREADS / 64];
  constexpr int T = SWEEP_THREADS;
  const int n = a.F.n, m = a.m, t = threadIdx.x;
  // own[0..2][n]: round r reads own[r % 3] (blocked(k) = own < i), claims into own[(r + 1) % 3] and
  // resets own[(r + 2) % 3] from base[n] = -1 for a taken keypoint (pre-blocked or claimed by an
  // earlier chunk: every such query index is smaller than the chunk's), INT_MAX otherwise
  int* ownb = s_lds;
  int* base = ownb + 3 * n;
  int* list = base + n;
  for (int k = t; k < n; k += T) {
    const int b0 = sbp_pre_blocked(a, k) ? -1 : INT_MAX;
    base[k] = b0;
    ownb[k] = b0;
    ownb[n + k] = b0;
    ownb[2 * n + k] = b0;
  }
  __syncthreads();
  const int C = s.chunk, mwords = (m + 31) >> 5;
  int len = 0, n_chunks = 0, n_rounds = 0, n_live = 0, n_seq = 0, max_r = 0, n_over = 0;
  // phase clock (thread 0, 100 MHz wall clock): [0] compaction, [1] the chunks' loads, [2] their
  // rounds, [3] their commits
  unsigned long long tck[4] = {0, 0, 0, 0}, tlast = t == 0 ? wall_clock64() : 0;
  const unsigned long long wall0 = tlast, cyc0 = t == 0 ? clock64() : 0;  // (the shader clock's rate)
  auto tick = [&](int ph) {
    if (t == 0) {
      const unsigned long long now = wall_clock64();
      tck[ph] += now - tlast;
      tlast = now;
    }
  };
  for (int w0 = 0; w0 < mwords; w0 += SWEEP_WINDOW_WORDS) {
    // this window's live queries appended to the list in ascending order (thread t: bitmap word w0 + t)
    const int wi = w0 + t;
    uint32_t bits = t < SWEEP_WINDOW_WORDS && wi < mwords ? a.live[wi] : 0u;
    int total;
    int pos = len + sweep_scan_incl(__popc(bits), s_wsum, &total) - __popc(bits);
    while (bits) {
      list[pos++] = 32 * wi + __builtin_ctz(bits);
      bits &= bits - 1u;
    }
    len += total;
    n_live += total;
    __syncthreads();
    tick(0);
    const bool last = w0 + SWEEP_WINDOW_WORDS >= mwords;
    int c0 = 0;
    while (len - c0 >= C || (last && c0 < len)) {
      // ---- one chunk: thread t <-> live query c0 + t, its count, flags and first SWEEP_E cache
      //      entries in registers (loaded together) ----
      const int cn = min(C, len - c0);
      const int i = t < cn ? list[c0 + t] : -1;
      int nq = 0, fl = 0;
      uint32_t e[SWEEP_E];
      const uint32_t* ce = nullptr;
      if (i >= 0) {
        ce = a.cand + (size_t)i * a.cand_cap;
#pragma unroll
        for (int u = 0; u < SWEEP_E; u++) e[u] = u < a.cand_cap ? ce[u] : 0u;  // (stale past cand_n: unused)
        nq = a.cand_n[i];
        fl = a.q[i].flags;
      }
      tick(1);
      int res = INT_MIN, r = 0;
      bool seq = false;
      for (;; r++) {
        if (r >= s.max_rounds) {
          seq = true;
          break;
        }
        const int* own_rd = ownb + (r % 3) * n;
        int* own_wr = ownb + ((r + 1) % 3) * n;
        int* own_clr = ownb + ((r + 2) % 3) * n;
        int nr = -1;
        if (i >= 0) {
          if (nq < 0) {  // more candidates than the cache holds: the grid walk
            nr = sbp_one(a, i, [&](int k) { return own_rd[k] < i; });
          } else {
            uint32_t k1 = 0xffffffffu, k2 = 0xffffffffu;
            int kk1 = -1;
            int ow[SWEEP_E];
#pragma unroll
            for (int u = 0; u < SWEEP_E; u++) ow[u] = u < nq ? own_rd[cand_key(e[u])] : INT_MAX;  // reads in flight together
#pragma unroll
            for (int u = 0; u < SWEEP_E; u++) {
              const uint32_t key = u < nq && ow[u] >= i ? sweep_key(e[u], u) : 0xffffffffu;
              k2 = min(k2, max(k1, key));
              kk1 = key < k1 ? cand_key(e[u]) : kk1;
              k1 = min(k1, key);
            }
            for (int u = SWEEP_E; u < nq; u++) {  // the rest from the cache (L2)
              const uint32_t x = ce[u];
              const uint32_t key = own_rd[cand_key(x)] >= i ? sweep_key(x, u) : 0xffffffffu;
              k2 = min(k2, max(k1, key));
              kk1 = key < k1 ? cand_key(x) : kk1;
              k1 = min(k1, key);
            }
            nr = sweep_result(a, k1, k2, kk1);
          }
        }
        if (i >= 0 && nr >= 0 && (fl & 2)) atomicMin(&own_wr[nr], i);  // (own_wr was reset last round)
        for (int k = t; k < n; k += T) own_clr[k] = base[k];  // next round's claim buffer
        const bool more = __syncthreads_or(i >= 0 && nr != res);
        if (!more) break;  // this round reproduced the last one
        res = nr;
      }
      tick(2);
      if (seq) {  // the reference loop over this chunk (debug knob only: C + 1 rounds always settle)
        __syncthreads();
        if (t == 0) {
          for (int c = 0; c < cn; c++) {
            const int qi = list[c0 + c];
            const int rr = sbp_eval(a, qi, [&](int k) { return base[k] < 0; });
            s.res[qi] = rr;
            if (rr >= 0 && (a.q[qi].flags & 2)) base[rr] = -1;
          }
          n_seq++;
        }
      } else if (i >= 0) {  // commit the chunk's claims
        s.res[i] = res;
        if (res >= 0 && (fl & 2)) base[res] = -1;
      }
      __syncthreads();
      // every owner buffer back to the base for the next chunk
      for (int k = t; k < n; k += T) {
        const int b0 = base[k];
        ownb[k] = b0;
        ownb[n + k] = b0;
        ownb[2 * n + k] = b0;
      }
      const int n_ov = __syncthreads_count(i >= 0 && nq < 0);
      tick(3);
      n_chunks++;
      n_over += n_ov;
      n_rounds += r;
      max_r = max(max_r, r);
      c0 += cn;
    }
    // the remainder (< C <= T entries) to the front of the list
    const int rem = len - c0;
    const int v = t < rem ? list[c0 + t] : 0;
    __syncthreads();
    if (t < rem) list[t] = v;
    __syncthreads();
    len = rem;
  }
  if (t == 0) {
    s.stats[1] = n_chunks;
    s.stats[2] = n_rounds;
    s.stats[3] = n_live;
    s.stats[4] = n_seq;
    s.stats[5] = max_r;
    for (int ph = 0; ph < 4; ph++) s.stats[6 + ph] = (int32_t)tck[ph];
    s.stats[10] = n_over;
    s.stats[11] = (int32_t)((clock64() - cyc0) / 1000);  // shader cycles / 1000 over the kernel
    s.stats[12] = (int32_t)(wall_clock64() - wall0);     // 100 MHz ticks over the kernel
    a.state[0] = 1;          // converged: k_sbp_collect / k_sbp_finish take the results
    a.state[1] = max_r + 1;  // (round statistics: round 0 + the deepest chunk)
    a.state[SBP_FINAL_SLOT] = 1;  // in round 0's buffer (res_final[0])
  }
}

struct SbpFinishArgs {
  SbpArgs s;
  const int32_t* res_final[2];  // result buffers by round parity
  int32_t* best_out;
  int32_t* nmatches;
  int check_ori;
  const float* q_angle;  // last-frame keypoint angles (mode 1)
  int32_t* serial_used;  // 1: the serial walk ran; 2: unsettled, deferred to more rounds
  int defer;
};

// Sequential fallback (the reference loop verbatim) when the fixpoint did not settle in
// SBP_MAX_ROUNDS rounds, then counting and (last frame) the rotation-consistency filter.
__device__ __forceinline__ bool sbp_converged(const SbpArgs& a) {
  // settled: a round was skipped, or the last round reproduced the round before it
  const int rounds = a.state[1];
  return a.state[0] != 0 || (rounds >= 2 && a.state[2 + rounds - 1] == 0);
}

// The final results: round state[1]-1's buffer, or the one k_sbp_sweep updated in place.
__device__ __forceinline__ const int32_t* sbp_final(const SbpFinishArgs& f) {
  const int slot = f.s.state[SBP_FINAL_SLOT];
  return slot ? f.res_final[slot - 1] : f.res_final[(f.s.state[1] - 1) & 1];
}

// Converged without a rotation filter (the local search): results and count, grid-wide.
__global__ __launch_bounds__(256) void k_sbp_collect(SbpFinishArgs f) {
  const SbpArgs& a = f.s;
  if (f.check_ori || !sbp_converged(a)) return;  // k_sbp_finish handles those
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int32_t* res = sbp_final(f);
  int c = 0;
  if (i < a.m) {
    const int r = res[i];
    f.best_out[i] = r;
    c = r >= 0;
  }
  // one atomic per block (same-address device atomics serialise across the XCDs)
  __shared__ int s_c[4];
  c = wave_sum(c);
  if (lane_id() == 0) s_c[wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0 && s_c[0] + s_c[1] + s_c[2] + s_c[3]) atomicAdd(f.nmatches, s_c[0] + s_c[1] + s_c[2] + s_c[3]);
}

__global__ __launch_bounds__(256) void k_sbp_finish(SbpFinishArgs f, int32_t* blocked_scratch) {
  __shared__ int s_hist[HISTO_LENGTH];
  __shared__ int s_misc[8];
  const SbpArgs& a = f.s;
  const int t = threadIdx.x;
  const bool converged = sbp_converged(a);
  if (converged && !f.check_ori) return;  // done by k_sbp_collect
  const int32_t* res = sbp_final(f);
  if (!converged && f.defer) {  // the host continues the rounds (sbp_fetch)
    if (t == 0) *f.serial_used = 2;
    return;
  }
  if (!converged) {
    if (t == 0) {
      *f.serial_used = 1;
      for (int k = 0; k < a.F.n; k++) blocked_scratch[k] = sbp_pre_blocked(a, k);
      for (int i = 0; i < a.m; i++) {
        const int r = sbp_one(a, i, [&](int k) { return blocked_scratch[k] != 0; });
        f.best_out[i] = r;
        if (r >= 0) blocked_scratch[r] = (a.q[i].flags & 2) ? 1 : 0;
      }
    }
    __syncthreads();
    __threadfence_block();
  } else {
    for (int i = t; i < a.m; i += 256) f.best_out[i] = res[i];
    __syncthreads();
  }
  if (t < HISTO_LENGTH) s_hist[t] = 0;
  if (t == 0) s_misc[4] = 0;
  __syncthreads();
  if (f.check_ori) {
    for (int i = t; i < a.m; i += 256) {
      const int b = f.best_out[i];
      if (b >= 0) atomicAdd(&s_hist[rot_bin_dev(f.q_angle[i], a.F.keys_un[b].angle)], 1);
    }
    __syncthreads();
    if (t == 0) three_maxima_dev(s_hist, s_misc[0], s_misc[1], s_misc[2]);
    __syncthreads();
  }
  int cnt = 0;
  for (int i = t; i < a.m; i += 256) {
    const int b = f.best_out[i];
    if (b < 0) continue;
    if (f.check_ori) {
      const int bin = rot_bin_dev(f.q_angle[i], a.F.keys_un[b].angle);
      if (bin != s_misc[0] && bin != s_misc[1] && bin != s_misc[2]) {
        f.best_out[i] = -2 - b;  // assigned, then undone by the rotation filter
        continue;
      }
    }
    cnt++;
  }
  cnt = wave_sum(cnt);
  if (lane_id() == 0) atomicAdd(&s_misc[4], cnt);
  __syncthreads();
  if (t == 0) *f.nmatches = s_misc[4];
}

// Queries of SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:51-73)
struct LocalQueryArgs {
  orbfe_local_mappoints mp;  // device pointers
  const float* scale_factors;
  float th;
  SbpQuery* q;
};
__global__ void k_sbp_local_queries(LocalQueryArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.mp.m) return;
  SbpQuery q = {};
  const uint8_t fl = a.mp.flags[i];
  if ((fl & ORBFE_MPF_TRACK_IN_VIEW) && !(fl & ORBFE_MPF_BAD)) {
    const int lvl = a.mp.level[i];
    float r = a.mp.view_cos[i] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:135-141)
    if (a.th != 1.0) r *= a.th;
    q.x = a.mp.proj_x[i];
    q.y = a.mp.proj_y[i];
    q.r = r * a.scale_factors[lvl];
    q.xr = a.mp.proj_xr[i];
    q.er_lim = r * a.scale_factors[lvl];
    q.min_level = lvl - 1;
    q.max_level = lvl;
    q.flags = 1 | ((fl & ORBFE_MPF_OBSERVED) ? 2 : 0);
  }
  a.q[i] = q;
}

// Frame::isInFrustum (Frame.cc:318-374) + PredictScale (MapPoint.cc:432-447), thread per
// MapPoint; skip rules of Tracking::SearchLocalPoints (Tracking.cc:1193-1196).
struct FrustumArgs {
  int m;
  const uint8_t* flags_in;
  const float* pos;
  const float* normal;
  const float* min_d;
  const float* max_d;
  orbfe_frustum_out out;  // device pointers (all set)
  int32_t* n_in_view;     // device counter (zeroed before the launch)
  float rcw[9], tcw[3], ow[3];
  float fx, fy, cx, cy, bf, min_x, max_x, min_y, max_y;
  float cos_limit;
  int nlevels;
  float scale_thr[ORBFE_MAX_LEVELS_M];  // PredictScale table (predict_scale_table)
};
__global__ __launch_bounds__(256) void k_frustum(FrustumArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool in = false;
  if (i < a.m) {
    const uint8_t fl = (uint8_t)(a.flags_in[i] & ~ORBFE_MPF_TRACK_IN_VIEW);  // :320
    float u = 0.f, v = 0.f, xr = 0.f, viewCos = 0.f;
    int nScale = 0;
    if (!(fl & (ORBFE_MPF_BAD | ORBFE_MPF_SEEN))) {
      const float Px = a.pos[3 * i], Py = a.pos[3 * i + 1], Pz = a.pos[3 * i + 2];
      const float PcX = gemv3_d(a.rcw, Px, Py, Pz, a.tcw[0]);
      const float PcY = gemv3_d(a.rcw + 3, Px, Py, Pz, a.tcw[1]);
      const float PcZ = gemv3_d(a.rcw + 6, Px, Py, Pz, a.tcw[2]);
      if (!(PcZ < 0.0f)) {
        const float invz = 1.0f / PcZ;
        u = a.fx * PcX * invz + a.cx;
        v = a.fy * PcY * invz + a.cy;
        if (!(u < a.min_x || u > a.max_x) && !(v < a.min_y || v > a.max_y)) {
          const float maxDistance = 1.2f * a.max_d[i];
          const float minDistance = 0.8f * a.min_d[i];
          const float POx = Px - a.ow[0], POy = Py - a.ow[1], POz = Pz - a.ow[2];
          double ss = (double)POx * (double)POx;  // cv::norm (:350)
          ss += (double)POy * (double)POy;
          ss += (double)POz * (double)POz;
          const float dist = (float)sqrt(ss);
          if (!(dist < minDistance || dist > maxDistance)) {
            double dot = (double)POx * (double)a.normal[3 * i];  // Mat::dot (:358)
            dot += (double)POy * (double)a.normal[3 * i + 1];
            dot += (double)POz * (double)a.normal[3 * i + 2];
            viewCos = (float)(dot / (double)dist);
            if (!(viewCos < a.cos_limit)) {
              nScale = predict_scale_dev(a.max_d[i], dist, a.scale_thr, a.nlevels);
              xr = u - a.bf * invz;
              in = true;
            }
          }
        }
      }
    }
    a.out.flags[i] = (uint8_t)(fl | (in ? ORBFE_MPF_TRACK_IN_VIEW : 0u));
    if (in) {
      a.out.proj_x[i] = u;
      a.out.proj_y[i] = v;
      a.out.proj_xr[i] = xr;
      a.out.level[i] = nScale;
      a.out.view_cos[i] = viewCos;
    }
  }
  __shared__ int s_n[4];  // one atomic per block (same-address device atomics serialise)
  const uint64_t b = wave_ballot(in);
  if (lane_id() == 0) s_n[wave_id()] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0 && s_n[0] + s_n[1] + s_n[2] + s_n[3]) atomicAdd(a.n_in_view, s_n[0] + s_n[1] + s_n[2] + s_n[3]);
}

// Queries of SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:1358-1410):
// projection with cv::Mat float algebra accumulated in double.
struct LastQueryArgs {
  orbfe_lastframe_mappoints last;  // device pointers
  orbfe_frame_view C;              // camera + level tables (device pointers)
  float rcw[9], tcw[3];
  int forward, backward;
  float th;
  SbpQuery* q;
};
__device__ __forceinline__ float gemv_row_dev(const float* r, const float* v, float add) {
  double s = (double)r[0] * (double)v[0];
  s += (double)r[1] * (double)v[1];
  s += (double)r[2] * (double)v[2];
  s = s + (double)add;
  return (float)s;
}
__global__ void k_sbp_last_queries(LastQueryArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.last.n) return;
  SbpQuery q = {};
  const uint8_t fl = a.last.flags[i];
  if ((fl & ORBFE_MPF_PRESENT) && !(fl & ORBFE_MPF_OUTLIER)) {
    const float X[3] = {a.last.world_pos[3 * i], a.last.world_pos[3 * i + 1], a.last.world_pos[3 * i + 2]};
    const float xc = gemv_row_dev(a.rcw, X, a.tcw[0]);
    const float yc = gemv_row_dev(a.rcw + 3, X, a.tcw[1]);
    const float zc = gemv_row_dev(a.rcw + 6, X, a.tcw[2]);
    const float invzc = (float)(1.0 / (double)zc);
    const float u = a.C.fx * xc * invzc + a.C.cx;
    const float v = a.C.fy * yc * invzc + a.C.cy;
    if (!(invzc < 0) && !(u < a.C.min_x || u > a.C.max_x) && !(v < a.C.min_y || v > a.C.max_y)) {
      const int oct = a.last.octave[i];
      const float radius = a.th * a.C.scale_factors[oct];
      q.x = u;
      q.y = v;
      q.r = radius;
      q.xr = u - a.C.bf * invzc;
      q.er_lim = radius;
      if (a.forward) { q.min_level = oct; q.max_level = -1; }
      else if (a.backward) { q.min_level = 0; q.max_level = oct; }
      else { q.min_level = oct - 1; q.max_level = oct + 1; }
      q.flags = 1 | ((fl & ORBFE_MPF_OBSERVED) ? 2 : 0);
    }
  }
  a.q[i] = q;
}

__global__ void k_hamming_batch(const uint8_t* a, const uint8_t* b, int n, int32_t* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint4 a0, a1, b0, b1;
  load_desc(a + (size_t)i * 32, a0, a1);
  load_desc(b + (size_t)i * 32, b0, b1);
  out[i] = hamming256(a0, a1, b0, b1);
}

// =============================================================================================
// host side
namespace orbfe_mi {
int ensure_arena(orbfe_matcher* m, size_t bytes) {
  m->stage_lo = SIZE_MAX;
  m->stage_hi = 0;
  m->d2d.clear();
  m->d2h.clear();
  if (bytes > m->arena_bytes) {
    hipFree(m->arena);
    m->arena = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&m->arena, bytes));
    m->arena_bytes = bytes;
  }
  if (bytes > m->pinned_bytes) {
    if (m->pinned) hipHostFree(m->pinned);
    m->pinned = nullptr;
    ORBFE_HIP_CHECK(hipHostMalloc((void**)&m->pinned, bytes, hipHostMallocDefault));
    m->pinned_bytes = bytes;
  }
  return ORBFE_OK;
}

// Stage n host bytes for arena address dst (uploaded by flush_h2d).
// A caller's array in device memory (a resident local map, a frame left in HBM): hipMemcpyAsync
// device to device instead of the host staging copy. Pageable host memory reports
// hipMemoryTypeUnregistered or an error, which is cleared here.
// An error an earlier call left pending on this thread is taken out first and reported by the
// next flush_h2d, so the query's own cleanup cannot swallow it.
static bool is_device_ptr(orbfe_matcher* m, const void* p) {
  const hipError_t prior = hipGetLastError();
  if (prior != hipSuccess && m->pending_err == hipSuccess) m->pending_err = prior;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice;
}

void stage_h2d(orbfe_matcher* m, const void* dst, const void* src, size_t n) {
  if (n == 0) return;
  const size_t off = (size_t)((const uint8_t*)dst - m->arena);
  if (is_device_ptr(m, src)) {
    m->d2d.emplace_back(off, src, n);
    return;
  }
  std::memcpy(m->pinned + off, src, n);
  m->stage_lo = std::min(m->stage_lo, off);
  m->stage_hi = std::max(m->stage_hi, off + n);
}

// One H2D copy of the staged span (arena regions in between are written by kernels afterwards).
int flush_h2d(orbfe_matcher* m) {
  if (m->pending_err != hipSuccess) {
    const hipError_t e = m->pending_err;
    m->pending_err = hipSuccess;
    m->stage_lo = SIZE_MAX;
    m->stage_hi = 0;
    m->d2d.clear();
    return orbfe_set_hip_error(e, "an earlier HIP call (pending before this search)");
  }
  if (m->stage_hi > m->stage_lo)
    ORBFE_HIP_CHECK(hipMemcpyAsync(m->arena + m->stage_lo, m->pinned + m->stage_lo, m->stage_hi - m->stage_lo,
                                   hipMemcpyHostToDevice, m->stream));
  m->stage_lo = SIZE_MAX;
  m->stage_hi = 0;
  for (const auto& c : m->d2d)
    ORBFE_HIP_CHECK(hipMemcpyAsync(m->arena + std::get<0>(c), std::get<1>(c), std::get<2>(c),
                                   hipMemcpyDeviceToDevice, m->stream));
  m->d2d.clear();
  return ORBFE_OK;
}

void stage_d2h(orbfe_matcher* m, void* dst, const void* src, size_t n) {
  if (n == 0 || !dst) return;
  m->d2h.emplace_back(dst, (size_t)((const uint8_t*)src - m->arena), n);
}

int fetch_d2h(orbfe_matcher* m) {
  size_t lo = SIZE_MAX, hi = 0, sum = 0;
  for (const auto& r : m->d2h) {
    lo = std::min(lo, std::get<1>(r));
    hi = std::max(hi, std::get<1>(r) + std::get<2>(r));
    sum += std::get<2>(r);
  }
  const bool span = !m->d2h.empty() && m->pinned && hi <= m->pinned_bytes && hi - lo <= 4 * sum + (64u << 10);
  int st = ORBFE_OK;
  if (span) {
    if (hipMemcpyAsync(m->pinned + lo, m->arena + lo, hi - lo, hipMemcpyDeviceToHost, m->stream) != hipSuccess)
      st = orbfe_set_error(ORBFE_ERR_HIP, "fetch_d2h: hipMemcpyAsync");
  } else {
    for (const auto& r : m->d2h)
      if (st == ORBFE_OK && hipMemcpyAsync(std::get<0>(r), m->arena + std::get<1>(r), std::get<2>(r),
                                           hipMemcpyDeviceToHost, m->stream) != hipSuccess)
        st = orbfe_set_error(ORBFE_ERR_HIP, "fetch_d2h: hipMemcpyAsync");
  }
  if (hipStreamSynchronize(m->stream) != hipSuccess && st == ORBFE_OK)
    st = orbfe_set_error(ORBFE_ERR_HIP, "fetch_d2h: hipStreamSynchronize");
  if (span && st == ORBFE_OK)
    for (const auto& r : m->d2h) std::memcpy(std::get<0>(r), m->pinned + std::get<1>(r), std::get<2>(r));
  m->d2h.clear();
  return st;
}

// Layout of one frame view in the arena (FrameOffsets)
FrameOffsets plan_frame(Arena& ar, const orbfe_frame_view* f) {
  FrameOffsets o;
  o.keys = ar.add(sizeof(orbfe_keypoint) * std::max(f->n, 1));
  o.ur = ar.add(sizeof(float) * std::max(f->n, 1));
  o.desc = ar.add(32 * (size_t)std::max(f->n, 1));
  o.mp = ar.add(std::max(f->n, 1));
  o.scale = ar.add(sizeof(float) * std::max(f->nlevels, 1));
  o.sigma2 = ar.add(sizeof(float) * std::max(f->nlevels, 1));
  return o;
}
int upload_frame(orbfe_matcher* m, const FrameOffsets& o, const orbfe_frame_view* f,
                 orbfe_frame_view* d) {
  uint8_t* A = m->arena;
  *d = *f;
  d->keys_un = (const orbfe_keypoint*)(A + o.keys);
  d->u_right = (const float*)(A + o.ur);
  d->descriptors = A + o.desc;
  d->mp_state = A + o.mp;
  d->scale_factors = (const float*)(A + o.scale);
  d->level_sigma2 = (const float*)(A + o.sigma2);
  if (f->n > 0) {
    stage_h2d(m, A + o.keys, f->keys_un, sizeof(orbfe_keypoint) * f->n);
    stage_h2d(m, A + o.ur, f->u_right, sizeof(float) * f->n);
    stage_h2d(m, A + o.desc, f->descriptors, 32 * (size_t)f->n);
    stage_h2d(m, A + o.mp, f->mp_state, f->n);
  }
  if (f->nlevels > 0) {
    stage_h2d(m, A + o.scale, f->scale_factors, sizeof(float) * f->nlevels);
    if (f->level_sigma2) stage_h2d(m, A + o.sigma2, f->level_sigma2, sizeof(float) * f->nlevels);
  }
  return ORBFE_OK;
}
bool frame_ok(const orbfe_frame_view* f) {
  return f && f->n >= 0 && f->n <= GRID_MAX_KEYS && (f->n == 0 || (f->keys_un && f->u_right && f->descriptors && f->mp_state)) &&
         f->nlevels > 0 && f->nlevels <= ORBFE_MAX_LEVELS_M && f->scale_factors;
}
bool levels_ok(const orbfe_keypoint* k, int n, int nlevels) {
  for (int i = 0; i < n; i++)
    if (k[i].octave < 0 || k[i].octave >= nlevels) return false;
  return true;
}
}  // namespace

extern "C" int orbfe_matcher_create(float nnratio, int check_orientation, int device,
                                    orbfe_matcher** out) {
  if (!out) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_matcher_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_matcher_create: no HIP device");
  if (device < 0 || device >= ndev) return orbfe_set_error(ORBFE_ERR_ARG, "bad device index");
  orbfe_matcher* m = new orbfe_matcher();
  m->device = device;
  m->nnratio = nnratio;
  m->check_ori = check_orientation ? 1 : 0;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&m->d_serial, sizeof(int32_t) * 16) != hipSuccess) {
    delete m;
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_matcher_create: HIP setup failed");
  }
  *out = m;
  return ORBFE_OK;
}

extern "C" int orbfe_matcher_destroy(orbfe_matcher* m) {
  if (!m) return ORBFE_OK;
  hipSetDevice(m->device);
  if (m->stream) hipStreamSynchronize(m->stream);
  hipFree(m->arena);
  hipFree(m->d_pairs);
  hipFree(m->d_serial);
  if (m->stream) hipStreamDestroy(m->stream);
  if (m->prof_ev0) hipEventDestroy(m->prof_ev0);
  if (m->prof_ev1) hipEventDestroy(m->prof_ev1);
  delete m;
  return ORBFE_OK;
}

extern "C" void* orbfe_matcher_stream(orbfe_matcher* m) { return m ? (void*)m->stream : nullptr; }

extern "C" int orbfe_matcher_set_profiling(orbfe_matcher* m, int on) {
  if (!m) return ORBFE_ERR_ARG;
  hipSetDevice(m->device);
  if (on && !m->prof_ev0) {
    ORBFE_HIP_CHECK(hipEventCreate(&m->prof_ev0));
    ORBFE_HIP_CHECK(hipEventCreate(&m->prof_ev1));
  }
  m->profile = on ? 1 : 0;
  m->prof_started = m->prof_done = false;
  return ORBFE_OK;
}

extern "C" int orbfe_matcher_last_device_ms(orbfe_matcher* m, float* ms) {
  if (!m || !ms) return ORBFE_ERR_ARG;
  if (!m->profile || !m->prof_done) return orbfe_set_error(ORBFE_ERR_STATE, "no profiled call yet");
  ORBFE_HIP_CHECK(hipEventSynchronize(m->prof_ev1));
  ORBFE_HIP_CHECK(hipEventElapsedTime(ms, m->prof_ev0, m->prof_ev1));
  return ORBFE_OK;
}

extern "C" int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  if (!a || !b) return ORBFE_ERR_ARG;
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

extern "C" int orbfe_descriptor_distance_batch(orbfe_matcher* m, const uint8_t* a,
                                               const uint8_t* b, int n, int32_t* out) {
  if (!m || n < 0 || (n > 0 && (!a || !b || !out))) return ORBFE_ERR_ARG;
  if (n == 0) return ORBFE_OK;
  hipSetDevice(m->device);
  Arena ar;
  const size_t oa = ar.add(32 * (size_t)n), ob = ar.add(32 * (size_t)n), oo = ar.add(4 * (size_t)n);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  ORBFE_HIP_CHECK(hipMemcpyAsync(m->arena + oa, a, 32 * (size_t)n, hipMemcpyHostToDevice, m->stream));
  ORBFE_HIP_CHECK(hipMemcpyAsync(m->arena + ob, b, 32 * (size_t)n, hipMemcpyHostToDevice, m->stream));
  ORBFE_LAUNCH("k_hamming_batch", k_hamming_batch, dim3((n + 255) / 256), dim3(256), 0, m->stream, m->arena + oa,
                     m->arena + ob, n, (int32_t*)(m->arena + oo));
  ORBFE_HIP_CHECK(hipGetLastError());
  ORBFE_HIP_CHECK(hipMemcpyAsync(out, m->arena + oo, 4 * (size_t)n, hipMemcpyDeviceToHost, m->stream));
  ORBFE_HIP_CHECK(hipStreamSynchronize(m->stream));
  return ORBFE_OK;
}

// ---- SearchForTriangulation ---------------------------------------------------------------
extern "C" int orbfe_search_for_triangulation_batch_device(orbfe_matcher* m, int n_pairs,
                                                           const orbfe_sft_pair* pairs,
                                                           int only_stereo, void* stream) {
  if (!m || n_pairs < 0 || (n_pairs > 0 && !pairs)) return orbfe_set_error(ORBFE_ERR_ARG, "sft batch: bad argument");
  if (n_pairs == 0) return ORBFE_OK;
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  if (n_pairs > m->pairs_cap) {
    hipFree(m->d_pairs);
    m->d_pairs = nullptr;
    m->pairs_uploaded.clear();
    ORBFE_HIP_CHECK(hipMalloc(&m->d_pairs, sizeof(orbfe_sft_pair) * n_pairs));
    m->pairs_cap = n_pairs;
  }
  for (int p = 0; p < n_pairs; p++)
    if (pairs[p].kf2.n > SFT_MAX_KF2) return orbfe_set_error(ORBFE_ERR_ARG, "sft: KF2 too large");
  // the pair descriptors are usually identical from call to call (device-resident batches):
  // upload only when they changed
  if ((int)m->pairs_uploaded.size() != n_pairs ||
      std::memcmp(m->pairs_uploaded.data(), pairs, sizeof(orbfe_sft_pair) * n_pairs) != 0) {
    ORBFE_HIP_CHECK(hipMemcpyAsync(m->d_pairs, pairs, sizeof(orbfe_sft_pair) * n_pairs, hipMemcpyHostToDevice, s));
    m->pairs_uploaded.assign(pairs, pairs + n_pairs);
  }
  // fv1.n_nodes bounds the node grid (with fv1_nodes_dev set it must be an upper bound)
  int max_nodes = 1;
  for (int p = 0; p < n_pairs; p++) max_nodes = std::max(max_nodes, pairs[p].fv1.n_nodes);
  // (max_nodes + 3) / 4 workgroups of node wavefronts + one for the features no node lists +
  // SFT_BIG_WG for the nodes past the wavefront fixpoint
  ORBFE_LAUNCH("k_sft_nodes", k_sft_nodes, dim3((max_nodes + 3) / 4 + 1 + SFT_BIG_WG, n_pairs), dim3(256), 0, s,
               m->d_pairs,
                     only_stereo ? 1 : 0);
  ORBFE_LAUNCH("k_sft_finish", k_sft_finish, dim3(n_pairs), dim3(256), 0, s, m->d_pairs, m->check_ori);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

extern "C" int orbfe_search_for_triangulation(orbfe_matcher* m, const orbfe_frame_view* kf1,
                                              const orbfe_frame_view* kf2,
                                              const orbfe_feature_vector* fv1,
                                              const orbfe_feature_vector* fv2, const float* f12,
                                              float ex, float ey, int only_stereo,
                                              int32_t* match12, int* nmatches) {
  if (!m || !frame_ok(kf1) || !frame_ok(kf2) || !fv1 || !fv2 || !f12 || !nmatches ||
      (kf1->n > 0 && !match12) || !kf2->level_sigma2)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_for_triangulation: bad argument");
  if (!levels_ok(kf2->keys_un, kf2->n, kf2->nlevels))
    return orbfe_set_error(ORBFE_ERR_ARG, "keypoint octave outside the level tables");
  hipSetDevice(m->device);
  Arena ar;
  const FrameOffsets o1 = plan_frame(ar, kf1), o2 = plan_frame(ar, kf2);
  auto plan_fv = [&](const orbfe_feature_vector* fv, size_t* ids, size_t* offs, size_t* idx) {
    *ids = ar.add(4 * (size_t)std::max(fv->n_nodes, 1));
    *offs = ar.add(4 * (size_t)(fv->n_nodes + 1));
    *idx = ar.add(4 * (size_t)std::max(fv->n_nodes > 0 ? fv->offsets[fv->n_nodes] : 0, 1));
  };
  size_t f1i, f1o, f1x, f2i, f2o, f2x;
  plan_fv(fv1, &f1i, &f1o, &f1x);
  plan_fv(fv2, &f2i, &f2o, &f2x);
  const size_t om = ar.add(4 * (size_t)std::max(kf1->n, 1)), on = ar.add(4);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  orbfe_sft_pair P;
  std::memset(&P, 0, sizeof(P));
  if ((st = upload_frame(m, o1, kf1, &P.kf1))) return st;
  if ((st = upload_frame(m, o2, kf2, &P.kf2))) return st;
  auto up_fv = [&](const orbfe_feature_vector* fv, size_t ids, size_t offs, size_t idx,
                   orbfe_feature_vector* d) -> int {
    uint8_t* A = m->arena;
    d->n_nodes = fv->n_nodes;
    d->node_ids = (const uint32_t*)(A + ids);
    d->offsets = (const int32_t*)(A + offs);
    d->indices = (const int32_t*)(A + idx);
    if (fv->n_nodes > 0) {
      const int ni = fv->offsets[fv->n_nodes];
      stage_h2d(m, A + ids, fv->node_ids, 4 * (size_t)fv->n_nodes);
      stage_h2d(m, A + offs, fv->offsets, 4 * (size_t)(fv->n_nodes + 1));
      if (ni > 0) stage_h2d(m, A + idx, fv->indices, 4 * (size_t)ni);
    }
    return ORBFE_OK;
  };
  if ((st = up_fv(fv1, f1i, f1o, f1x, &P.fv1))) return st;
  if ((st = up_fv(fv2, f2i, f2o, f2x, &P.fv2))) return st;
  std::memcpy(P.f12, f12, sizeof(float) * 9);
  P.ex = ex;
  P.ey = ey;
  P.match12 = (int32_t*)(m->arena + om);
  P.nmatches = (int32_t*)(m->arena + on);
  if ((st = flush_h2d(m))) return st;
  st = orbfe_search_for_triangulation_batch_device(m, 1, &P, only_stereo, m->stream);
  if (st) return st;
  int32_t nm = 0;
  if (kf1->n > 0) orbfe_mi::stage_d2h(m, match12, P.match12, 4 * (size_t)kf1->n);
  orbfe_mi::stage_d2h(m, &nm, P.nmatches, 4);
  if ((st = orbfe_mi::fetch_d2h(m))) return st;
  *nmatches = nm;
  return ORBFE_OK;
}

// ---- SearchByProjection -----------------------------------------------------------------------
namespace orbfe_mi {
// host-staged inputs (frame, query descriptors / angles) ...
void sbp_plan_inputs(Arena& ar, const orbfe_frame_view* F, int nq, int cand_cap, SbpPlan& p) {
  p.nq = nq;
  p.cand_cap = cand_cap;
  p.fo = plan_frame(ar, F);
  const size_t q1 = (size_t)std::max(nq, 1);
  p.oqd = ar.add(32 * q1);
  p.oqa = ar.add(4 * q1);
}
// ... and device-only scratch, planned after every staged input of the call so that the staged
// bytes form one contiguous span (one H2D copy)
void sbp_plan_scratch(Arena& ar, const orbfe_frame_view* F, SbpPlan& p) {
  const size_t q1 = (size_t)std::max(p.nq, 1), f1 = (size_t)std::max(F->n, 1);
  const int cand_cap = p.cand_cap;
  p.og_start = ar.add(4 * (GRID_CELLS + 1));
  p.og_items = ar.add(16 * f1);
  p.oq = ar.add(sizeof(SbpQuery) * q1);
  p.ores0 = ar.add(4 * q1);
  p.ores1 = ar.add(4 * q1);
  p.oown0 = ar.add(4 * f1);
  p.oown1 = ar.add(4 * f1);
  p.oown2 = ar.add(4 * f1);
  p.oblk = ar.add(4 * f1);
  p.ostate = ar.add(4 * (SBP_ROUND_CAP + 4));
  p.obest = ar.add(4 * q1);
  p.onm = ar.add(4);  // (state, best, count adjacent: sbp_fetch takes them down in one copy)
  p.cache = F->n <= 65535;  // candidate keypoint indices are 16-bit (cand_pack)
  const size_t cq = p.cache ? (size_t)cand_cap * q1 : 0;
  p.ocand = ar.add(4 * cq);
  p.ocand_n = ar.add(p.cache ? 4 * q1 : 0);
  p.oown3 = ar.add(4 * f1);
  // k_sbp_sweep keeps own[n] and the taken bits of the frame's keypoints in LDS
  p.sweep = p.cache && p.nq > 0 && F->n <= SWEEP_MAX_KEYS;
  p.olive = ar.add(p.sweep ? 4 * ((q1 + 31) / 32) : 0);
}
int sbp_cand_cap(const orbfe_matcher* m) { return m->cand_cap > 0 ? m->cand_cap : SBP_CAND; }

// The distance from which a candidate can no longer decide a SearchByProjection result, whatever the
// claims (the sweep's round 0 leaves such candidates out of the cache). A result needs bestDist <=
// dist_th, so in first-minimum mode (1) only candidates within dist_th matter: a query whose
// smallest unblocked distance exceeds it gets -1 with or without the others. In mode 0 the ratio
// test (:122-129) also reads bestDist2: it rejects only if bestDist > nnratio * bestDist2 with
// bestDist <= dist_th, so a second-best d2 with nnratio * d2 >= dist_th (float, as the reference
// computes it) never rejects -- and neither does 256, the value d2 takes when such candidates are
// left out. The best candidate itself is within dist_th or the result is -1 either way.
static int sbp_keep_below(const SbpMode& md, float nnratio) {
  if (md.mode != 0) return std::min(256, md.dist_th + 1);
  if (!(nnratio > 0.f)) return 256;
  for (int d = std::max(md.dist_th + 1, 1); d < 256; d++)
    if (nnratio * (float)d >= (float)md.dist_th) return d;
  return 256;
}
SbpPlan sbp_plan(Arena& ar, const orbfe_frame_view* F, int nq, int cand_cap) {
  SbpPlan p;
  sbp_plan_inputs(ar, F, nq, cand_cap, p);
  sbp_plan_scratch(ar, F, p);
  return p;
}

int sbp_stage(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const uint8_t* h_qdesc,
              const float* h_qangle, orbfe_frame_view* dF) {
  uint8_t* A = m->arena;
  int st = upload_frame(m, p.fo, F, dF);
  if (st) return st;
  if (p.nq > 0) {
    if (h_qdesc) stage_h2d(m, A + p.oqd, h_qdesc, 32 * (size_t)p.nq);
    if (h_qangle) stage_h2d(m, A + p.oqa, h_qangle, 4 * (size_t)p.nq);
  }
  return ORBFE_OK;
}

static GridArgs grid_args(uint8_t* A, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF) {
  GridArgs g;
  g.keys = dF.keys_un;
  g.n = F->n;
  g.min_x = F->grid_origin_set ? F->grid_min_x : F->min_x;  // mGrid was built with these bounds
  g.min_y = F->grid_origin_set ? F->grid_min_y : F->min_y;
  g.inv_w = F->grid_inv_w;
  g.inv_h = F->grid_inv_h;
  g.start = (int32_t*)(A + p.og_start);
  g.recs = (uint4*)(A + p.og_items);
  g.u_right = dF.u_right;
  return g;
}

void sbp_launch_grid(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF) {
  const GridArgs g = grid_args(m->arena, p, F, dF);
  ORBFE_LAUNCH("k_grid", k_grid, dim3(1), dim3(1024), sizeof(int) * (GRID_CELLS + 1 + 16 + std::max(F->n, 1)),
                     m->stream, g);
}

static SbpArgs sbp_args(uint8_t* A, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
                        const SbpMode& md, float nnratio) {
  SbpArgs a;
  std::memset(&a, 0, sizeof(a));
  a.F = dF;
  a.grid_start = (const int32_t*)(A + p.og_start);
  a.grid_recs = (const uint4*)(A + p.og_items);
  a.q = (const SbpQuery*)(A + p.oq);
  a.qdesc = A + p.oqd;
  a.m = p.nq;
  a.mode = md.mode;
  a.nnratio = nnratio;
  a.dist_th = md.dist_th;
  a.block_any = md.block_any;
  a.cand_cap = p.cand_cap;
  a.no_claims = md.no_claims;
  a.keep_below = 256;
  a.state = (int32_t*)(A + p.ostate);
  if (p.cache) {
    a.cand = (uint32_t*)(A + p.ocand);
    a.cand_n = (int32_t*)(A + p.ocand_n);
  }
  (void)F;
  return a;
}

static void sbp_launch_init(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, bool sweep = false) {
  uint8_t* A = m->arena;
  SbpInit in;
  in.live = sweep ? (uint32_t*)(A + p.olive) : nullptr;
  in.res0 = (int32_t*)(A + p.ores0);
  in.res1 = (int32_t*)(A + p.ores1);
  in.own0 = (int32_t*)(A + p.oown0);
  in.own2 = (int32_t*)(A + p.oown3);  // round 0's owner_prev (read only without the cache)
  in.state = (int32_t*)(A + p.ostate);
  in.nmatches = (int32_t*)(A + p.onm);
  in.serial = m->d_serial;
  in.nq = std::max(p.nq, 1);
  in.nf = std::max(F->n, 1);
  const int nthreads = std::max(std::max(in.nq, in.nf), SBP_ROUND_CAP + 4);
  ORBFE_LAUNCH("k_sbp_init", k_sbp_init, dim3((nthreads + 255) / 256), dim3(256), 0, m->stream, in);
}

void sbp_launch_round0(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
                       const SbpMode& md) {
  uint8_t* A = m->arena;
  sbp_launch_grid(m, p, F, dF);
  sbp_launch_init(m, p, F);
  SbpArgs a = sbp_args(A, p, F, dF, md, m->nnratio);
  a.round = 0;
  a.res_cur = (int32_t*)(A + p.ores0);
  a.res_prev = (int32_t*)(A + p.ores1);
  a.owner_cur = (int32_t*)(A + p.oown0);
  a.owner_prev = (int32_t*)(A + p.oown3);
  a.owner_next = (int32_t*)(A + p.oown1);
  if (p.nq > 0)
    ORBFE_LAUNCH("k_sbp_round0", k_sbp_round0, dim3(std::max((p.nq + 15) / 16, (F->n + 255) / 256)), dim3(256), 0,
                       m->stream, a);
}

// Rounds r0 .. r1-1 of the fixpoint, then collect / finish (owner buffers rotate over four:
// round r claims into own[r % 4], reads own[(r + 3) % 4] (round r-1) and own[(r + 2) % 4]
// (round r-2), and clears own[(r + 1) % 4] for round r + 1, which nobody reads during round r).
// `settled`: the sweep ran (the claim order is complete on the device), so without a rotation
// filter k_sbp_finish has nothing to do.
static void sbp_finish_launch(orbfe_matcher* m, const SbpPlan& p, const SbpArgs& a, const SbpMode& md,
                              int32_t* const res_final[2], bool defer, bool settled = false) {
  uint8_t* A = m->arena;
  SbpFinishArgs f;
  std::memset(&f, 0, sizeof(f));
  f.s = a;
  f.res_final[0] = res_final[0];
  f.res_final[1] = res_final[1];
  f.best_out = (int32_t*)(A + p.obest);
  f.nmatches = (int32_t*)(A + p.onm);
  f.check_ori = md.check_ori;
  f.q_angle = (const float*)(A + p.oqa);
  f.serial_used = m->d_serial;
  f.defer = defer ? 1 : 0;
  if (!md.check_ori)  // (k_sbp_collect returns at once with the rotation filter)
    ORBFE_LAUNCH("k_sbp_collect", k_sbp_collect, dim3((p.nq + 255) / 256), dim3(256), 0, m->stream, f);
  if (md.check_ori || !settled)
    ORBFE_LAUNCH("k_sbp_finish", k_sbp_finish, dim3(1), dim3(256), 0, m->stream, f, (int32_t*)(A + p.oblk));
}

// Round 0 grid-wide (the candidate cache; queries that can never match pruned), then the claim
// order in k_sbp_sweep, then collect / finish: 4 launches after the grid whatever the depth of the
// claim order.
static void sbp_sweep_launch(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F,
                             const orbfe_frame_view& dF, const SbpMode& md) {
  uint8_t* A = m->arena;
  const int nq = p.nq;
  SbpArgs a = sbp_args(A, p, F, dF, md, m->nnratio);
  int32_t* res[2] = {(int32_t*)(A + p.ores0), (int32_t*)(A + p.ores1)};
  a.round = 0;
  a.res_cur = res[0];
  a.res_prev = res[1];
  a.owner_cur = (int32_t*)(A + p.oown0);
  a.owner_prev = (int32_t*)(A + p.oown3);
  a.owner_next = (int32_t*)(A + p.oown1);
  a.owner_rm2 = nullptr;
  a.prune = 1;
  a.live = (uint32_t*)(A + p.olive);
  a.keep_below = sbp_keep_below(md, m->nnratio);
  ORBFE_LAUNCH("k_sbp_round0", k_sbp_round0, dim3(std::max((nq + 15) / 16, (F->n + 255) / 256)), dim3(256), 0,
               m->stream, a);
  a.prune = 0;
  a.keep_below = 256;
  SbpSweepArgs sw;
  sw.res = res[0];
  sw.chunk = m->sweep_chunk > 0 ? std::min(m->sweep_chunk, SWEEP_THREADS) : SWEEP_THREADS;
  sw.max_rounds = m->sweep_max_rounds > 0 ? m->sweep_max_rounds : sw.chunk + 2;
  sw.stats = m->d_serial;
  ORBFE_LAUNCH("k_sbp_sweep", k_sbp_sweep, dim3(1), dim3(SWEEP_THREADS), sweep_lds(F->n), m->stream, a, sw);
  sbp_finish_launch(m, p, a, md, res, false, true);
}

static void sbp_rounds(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
                       const SbpMode& md, int r0, int r1, bool defer) {
  uint8_t* A = m->arena;
  const int nq = p.nq;
  SbpArgs a = sbp_args(A, p, F, dF, md, m->nnratio);
  int32_t* res[2] = {(int32_t*)(A + p.ores0), (int32_t*)(A + p.ores1)};
  int32_t* own[4] = {(int32_t*)(A + p.oown0), (int32_t*)(A + p.oown1), (int32_t*)(A + p.oown2),
                     (int32_t*)(A + p.oown3)};
  for (int r = r0; r < r1 && nq > 0; r++) {
    a.round = r;
    a.res_cur = res[r & 1];
    a.res_prev = res[(r + 1) & 1];
    a.owner_cur = own[r % 4];
    a.owner_prev = own[(r + 3) % 4];
    a.owner_next = own[(r + 1) % 4];
    // round r-2's owners: round r re-evaluates only the queries a keypoint whose owner changed
    // since can reach
    a.owner_rm2 = r >= 2 && p.cache ? own[(r + 2) % 4] : nullptr;
    if (r == 0 && p.cache)
      ORBFE_LAUNCH("k_sbp_round0", k_sbp_round0, dim3(std::max((nq + 15) / 16, (F->n + 255) / 256)), dim3(256), 0,
                         m->stream, a);
    else
      ORBFE_LAUNCH("k_sbp_round", k_sbp_round, dim3((std::max(nq, F->n) + 255) / 256), dim3(256), 0, m->stream, a);
  }
  if (nq > 0) sbp_finish_launch(m, p, a, md, res, defer);
}

// ORBFE_SBP_SWEEP=0: the claim order as grid-wide Jacobi rounds, one launch each, continued by
// the host (rounds 1-4's engine, for A/B)
static bool sbp_sweep_enabled() {
  static const bool on = !(std::getenv("ORBFE_SBP_SWEEP") && std::atoi(std::getenv("ORBFE_SBP_SWEEP")) == 0);
  return on;
}

int sbp_launch(orbfe_matcher* m, const SbpPlan& p, const orbfe_frame_view* F, const orbfe_frame_view& dF,
               const SbpMode& md, bool defer) {
  sbp_launch_grid(m, p, F, dF);
  // the sweep unless rounds are restricted (orbfe_matcher_set_max_rounds: the serial fallback's
  // tests) or no assignment blocks anything (one round is the result)
  bool sweep = p.sweep && !md.no_claims && m->round_cap >= SBP_MAX_ROUNDS && sbp_sweep_enabled();
  if (sweep && m->sweep_attr == 0) {
    // k_sbp_sweep's dynamic LDS (up to ~70 KiB) on this matcher's device, checked once per matcher
    // (one thread per matcher; the attribute is per device); refused: the grid-wide rounds instead
    const hipError_t e = hipFuncSetAttribute((const void*)k_sbp_sweep, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)sweep_lds(SWEEP_MAX_KEYS));
    m->sweep_attr = e == hipSuccess ? 1 : -1;
    if (e != hipSuccess) (void)hipGetLastError();
  }
  sweep = sweep && m->sweep_attr > 0;
  sbp_launch_init(m, p, F, sweep);
  m->sbp_deferred = false;
  m->sbp_swept = sweep;
  if (sweep) {
    sbp_sweep_launch(m, p, F, dF, md);
  } else {
    const int rounds = md.no_claims && p.cache ? 1 : m->max_rounds;
    m->sbp_deferred = defer && m->round_cap > rounds;
    sbp_rounds(m, p, F, dF, md, 0, rounds, m->sbp_deferred);
  }
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

int sbp_fetch(orbfe_matcher* m, const SbpPlan& p, int32_t* best_idx, int* nmatches, const orbfe_frame_view* F,
              const orbfe_frame_view* dF, const SbpMode* md) {
  uint8_t* A = m->arena;
  int32_t nm = 0, state[2] = {0, 0}, serial = 0;
  static const bool always_check = std::getenv("ORBFE_SBP_FETCH_SYNC") != nullptr;  // (A/B: the check every call)
  if (p.nq > 0 && F && dF && md && !(md->no_claims && p.cache) && (m->sbp_deferred || always_check)) {
    // a fixpoint still unsettled continues in doubling chunks of rounds (a rare case: one sync
    // per chunk), the serial walk only past round_cap. Only launches that deferred (the grid-wide
    // rounds with a round budget below round_cap) can leave it unsettled: after k_sbp_sweep, or
    // rounds whose k_sbp_finish walks the rest itself, this host round trip is skipped
    ORBFE_HIP_CHECK(hipMemcpyAsync(&serial, m->d_serial, 4, hipMemcpyDeviceToHost, m->stream));
    ORBFE_HIP_CHECK(hipStreamSynchronize(m->stream));
    int done = m->max_rounds;
    while (serial == 2) {
      const int next = std::min(std::max(2 * done, done + 1), m->round_cap);
      ORBFE_HIP_CHECK(hipMemsetAsync(m->d_serial, 0, 4, m->stream));
      sbp_rounds(m, p, F, *dF, *md, done, next, next < m->round_cap);
      ORBFE_HIP_CHECK(hipGetLastError());
      done = next;
      ORBFE_HIP_CHECK(hipMemcpyAsync(&serial, m->d_serial, 4, hipMemcpyDeviceToHost, m->stream));
      ORBFE_HIP_CHECK(hipStreamSynchronize(m->stream));
    }
  }
  // the device part ends after the last round (continuations included, with their host syncs)
  prof_end(m);
  // the round state, the results and the match count are adjacent in the arena (sbp_plan_scratch):
  // one copy into the pinned mirror at the same offsets, then host copies out (instead of three
  // copies, one of them into the caller's pageable array); the serial-walk flag only when a walk
  // could have run (k_sbp_sweep settles the claim order itself)
  static const bool split_copies = std::getenv("ORBFE_SBP_FETCH_SPLIT") != nullptr;  // (A/B: three copies)
  const bool one_copy =
      !split_copies && p.ostate < p.obest && p.obest < p.onm && m->pinned && p.onm + 4 <= m->pinned_bytes;
  if (p.nq > 0) {
    if (one_copy) {
      ORBFE_HIP_CHECK(hipMemcpyAsync(m->pinned + p.ostate, A + p.ostate, p.onm + 4 - p.ostate, hipMemcpyDeviceToHost,
                                     m->stream));
    } else {
      if (best_idx)
        ORBFE_HIP_CHECK(hipMemcpyAsync(best_idx, A + p.obest, 4 * (size_t)p.nq, hipMemcpyDeviceToHost, m->stream));
      ORBFE_HIP_CHECK(hipMemcpyAsync(&nm, A + p.onm, 4, hipMemcpyDeviceToHost, m->stream));
      ORBFE_HIP_CHECK(hipMemcpyAsync(state, A + p.ostate, 8, hipMemcpyDeviceToHost, m->stream));
    }
    if (!m->sbp_swept) ORBFE_HIP_CHECK(hipMemcpyAsync(&serial, m->d_serial, 4, hipMemcpyDeviceToHost, m->stream));
  }
  ORBFE_HIP_CHECK(hipStreamSynchronize(m->stream));
  if (p.nq > 0 && one_copy) {
    if (best_idx) std::memcpy(best_idx, m->pinned + p.obest, 4 * (size_t)p.nq);
    std::memcpy(&nm, m->pinned + p.onm, 4);
    std::memcpy(state, m->pinned + p.ostate, 8);
  }
  m->last_rounds = state[1];
  m->last_serial = serial;
  if (nmatches) *nmatches = nm;
  return ORBFE_OK;
}

// PredictScale's ceil(logf(ratio) / log_scale_factor) (MapPoint.cc:415-447, float overloads under
// `using namespace std`) is non-decreasing in ratio, so nScale >= k  <=>  ratio >= thr[k-1], the
// smallest float with ceilf(logf(thr) / lsf) >= k. Found by bisection over the ordered bit
// patterns of positive floats, with the host's own logf -- the device never evaluates a log.
void predict_scale_table(float lsf, int nlevels, float* thr) {
  auto level = [&](uint32_t bits) {
    float r;
    std::memcpy(&r, &bits, 4);
    return (int)std::ceil(std::log(r) / lsf);
  };
  for (int k = 1; k < nlevels; k++) {
    uint32_t lo = 1u, hi = 0x7f800000u;  // level(hi = +inf) is huge; level(lo) is very negative
    if (!(lsf > 0)) {                    // degenerate scale factor: nothing reaches level k
      thr[k - 1] = INFINITY;
      continue;
    }
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (level(mid) >= k) hi = mid;
      else lo = mid + 1;
    }
    std::memcpy(&thr[k - 1], &lo, 4);
  }
  for (int k = std::max(nlevels, 1); k < ORBFE_MAX_LEVELS_M; k++) thr[k - 1] = INFINITY;
}
}  // namespace orbfe_mi

extern "C" int orbfe_predict_scale_thresholds(float log_scale_factor, int nlevels, float* thresholds) {
  if (!thresholds || nlevels < 1 || nlevels > ORBFE_MAX_LEVELS_M)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_predict_scale_thresholds: bad argument");
  float t[ORBFE_MAX_LEVELS_M];
  predict_scale_table(log_scale_factor, nlevels, t);
  for (int k = 1; k < nlevels; k++) thresholds[k - 1] = t[k - 1];
  return ORBFE_OK;
}

static int run_sbp(orbfe_matcher* m, const orbfe_frame_view* F, int nq, const SbpMode& md,
                   const uint8_t* h_qdesc, const float* h_qangle,
                   const std::function<int(Arena&)>& plan_q,
                   const std::function<int(uint8_t*, const orbfe_frame_view&, SbpQuery*)>& make_q,
                   int32_t* best_idx, int* nmatches) {
  Arena ar;
  SbpPlan p;
  sbp_plan_inputs(ar, F, nq, sbp_cand_cap(m), p);
  plan_q(ar);
  sbp_plan_scratch(ar, F, p);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  uint8_t* A = m->arena;
  orbfe_frame_view dF;
  m->prof_started = m->prof_done = false;
  if ((st = sbp_stage(m, p, F, h_qdesc, h_qangle, &dF))) return st;
  if (nq > 0 && (st = make_q(A, dF, (SbpQuery*)(A + p.oq)))) return st;  // stages, flushes, builds queries
  if ((st = flush_h2d(m))) return st;
  prof_begin(m);  // (no-op when make_q's k_frustum already opened the window)
  if ((st = sbp_launch(m, p, F, dF, md, true))) return st;
  return sbp_fetch(m, p, best_idx, nmatches, F, &dF, &md);  // (closes the profiling window)
}

extern "C" int orbfe_search_by_projection_local(orbfe_matcher* m, const orbfe_frame_view* F,
                                                const orbfe_local_mappoints* mps, float th,
                                                int32_t* best_idx, int* nmatches) {
  if (!m || !frame_ok(F) || !mps || !nmatches || mps->m < 0 ||
      (mps->m > 0 && (!best_idx || !mps->flags || !mps->proj_x || !mps->proj_y || !mps->proj_xr ||
                      !mps->level || !mps->view_cos || !mps->descriptors)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_projection_local: bad argument");
  for (int i = 0; i < mps->m; i++)
    if ((mps->flags[i] & ORBFE_MPF_TRACK_IN_VIEW) && !(mps->flags[i] & ORBFE_MPF_BAD) &&
        (mps->level[i] < 0 || mps->level[i] >= F->nlevels))
      return orbfe_set_error(ORBFE_ERR_ARG, "mnTrackScaleLevel outside the level tables");
  hipSetDevice(m->device);
  size_t o_flags = 0, o_px = 0, o_py = 0, o_pxr = 0, o_lvl = 0, o_vc = 0;
  const int M = mps->m;
  auto plan = [&](Arena& ar) -> int {
    o_flags = ar.add(std::max(M, 1));
    o_px = ar.add(4 * (size_t)std::max(M, 1));
    o_py = ar.add(4 * (size_t)std::max(M, 1));
    o_pxr = ar.add(4 * (size_t)std::max(M, 1));
    o_lvl = ar.add(4 * (size_t)std::max(M, 1));
    o_vc = ar.add(4 * (size_t)std::max(M, 1));
    return 0;
  };
  auto make = [&](uint8_t* A, const orbfe_frame_view& dF, SbpQuery* dq) -> int {
    stage_h2d(m, A + o_flags, mps->flags, M);
    stage_h2d(m, A + o_px, mps->proj_x, 4 * (size_t)M);
    stage_h2d(m, A + o_py, mps->proj_y, 4 * (size_t)M);
    stage_h2d(m, A + o_pxr, mps->proj_xr, 4 * (size_t)M);
    stage_h2d(m, A + o_lvl, mps->level, 4 * (size_t)M);
    stage_h2d(m, A + o_vc, mps->view_cos, 4 * (size_t)M);
    int st = flush_h2d(m);
    if (st) return st;
    LocalQueryArgs qa;
    std::memset(&qa, 0, sizeof(qa));
    qa.mp.m = M;
    qa.mp.flags = A + o_flags;
    qa.mp.proj_x = (const float*)(A + o_px);
    qa.mp.proj_y = (const float*)(A + o_py);
    qa.mp.proj_xr = (const float*)(A + o_pxr);
    qa.mp.level = (const int32_t*)(A + o_lvl);
    qa.mp.view_cos = (const float*)(A + o_vc);
    qa.scale_factors = dF.scale_factors;
    qa.th = th;
    qa.q = dq;
    ORBFE_LAUNCH("k_sbp_local_queries", k_sbp_local_queries, dim3((M + 255) / 256), dim3(256), 0, m->stream, qa);
    return ORBFE_OK;
  };
  return run_sbp(m, F, M, SbpMode{0, TH_HIGH, 0, 0}, mps->descriptors, nullptr, plan, make, best_idx, nmatches);
}

extern "C" int orbfe_search_by_projection_lastframe(orbfe_matcher* m,
                                                    const orbfe_frame_view* C,
                                                    const orbfe_lastframe_mappoints* L,
                                                    const float* tcw_cur, float th, int mono,
                                                    int32_t* best_idx, int* nmatches) {
  if (!m || !frame_ok(C) || !L || !tcw_cur || !nmatches || L->n < 0 ||
      (L->n > 0 && (!best_idx || !L->flags || !L->world_pos || !L->descriptors || !L->octave || !L->angle)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_projection_lastframe: bad argument");
  for (int i = 0; i < L->n; i++)
    if ((L->flags[i] & ORBFE_MPF_PRESENT) && !(L->flags[i] & ORBFE_MPF_OUTLIER) &&
        (L->octave[i] < 0 || L->octave[i] >= C->nlevels))
      return orbfe_set_error(ORBFE_ERR_ARG, "last-frame octave outside the level tables");
  hipSetDevice(m->device);
  // twc = -Rcw.t() * tcw ; tlc = Rlw * twc + tlw (ORBmatcher.cc:1358-1369), double-accumulated
  const float* T = tcw_cur;
  const float Rcw[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
  const float tcw[3] = {T[3], T[7], T[11]};
  const float* Tl = L->tcw_last;
  float twc[3];
  for (int i = 0; i < 3; i++) {
    double s = (double)Rcw[i] * (double)tcw[0];
    s += (double)Rcw[3 + i] * (double)tcw[1];
    s += (double)Rcw[6 + i] * (double)tcw[2];
    twc[i] = -(float)s;
  }
  double s2 = (double)Tl[8] * (double)twc[0];
  s2 += (double)Tl[9] * (double)twc[1];
  s2 += (double)Tl[10] * (double)twc[2];
  s2 = s2 + (double)Tl[11];
  const float tlc2 = (float)s2;
  const bool fwd = tlc2 > C->b && !mono;
  const bool bwd = -tlc2 > C->b && !mono;
  const int N = L->n;
  size_t o_flags = 0, o_pos = 0, o_oct = 0;
  auto plan = [&](Arena& ar) -> int {
    o_flags = ar.add(std::max(N, 1));
    o_pos = ar.add(12 * (size_t)std::max(N, 1));
    o_oct = ar.add(4 * (size_t)std::max(N, 1));
    return 0;
  };
  auto make = [&](uint8_t* A, const orbfe_frame_view& dF, SbpQuery* dq) -> int {
    stage_h2d(m, A + o_flags, L->flags, N);
    stage_h2d(m, A + o_pos, L->world_pos, 12 * (size_t)N);
    stage_h2d(m, A + o_oct, L->octave, 4 * (size_t)N);
    int st = flush_h2d(m);
    if (st) return st;
    LastQueryArgs qa;
    std::memset(&qa, 0, sizeof(qa));
    qa.last.n = N;
    qa.last.flags = A + o_flags;
    qa.last.world_pos = (const float*)(A + o_pos);
    qa.last.octave = (const int32_t*)(A + o_oct);
    qa.C = dF;
    std::memcpy(qa.rcw, Rcw, sizeof(Rcw));
    std::memcpy(qa.tcw, tcw, sizeof(tcw));
    qa.forward = fwd;
    qa.backward = bwd;
    qa.th = th;
    qa.q = dq;
    ORBFE_LAUNCH("k_sbp_last_queries", k_sbp_last_queries, dim3((N + 255) / 256), dim3(256), 0, m->stream, qa);
    return ORBFE_OK;
  };
  return run_sbp(m, C, N, SbpMode{1, TH_HIGH, 0, m->check_ori}, L->descriptors, L->angle, plan, make, best_idx,
                 nmatches);
}

extern "C" int orbfe_matcher_set_max_rounds(orbfe_matcher* m, int rounds) {
  if (!m || rounds < 1 || rounds > SBP_MAX_ROUNDS) return ORBFE_ERR_ARG;
  m->max_rounds = rounds;
  m->round_cap = rounds;  // a fixed budget: the serial walk past it (tests of the fallback)
  return ORBFE_OK;
}

extern "C" int orbfe_debug_matcher_set_sweep(orbfe_matcher* m, int chunk, int max_rounds, int cand_cap) {
  if (!m || chunk < 0 || chunk > SWEEP_THREADS || max_rounds < 0 || cand_cap < 0 || cand_cap > 4096)
    return ORBFE_ERR_ARG;
  m->sweep_chunk = chunk;
  m->sweep_max_rounds = max_rounds;
  m->cand_cap = cand_cap;
  return ORBFE_OK;
}

extern "C" int orbfe_debug_matcher_sweep_stats(orbfe_matcher* m, int32_t* out12) {
  if (!m || !out12) return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipStreamSynchronize(m->stream));
  ORBFE_HIP_CHECK(hipMemcpy(out12, m->d_serial + 1, 12 * sizeof(int32_t), hipMemcpyDeviceToHost));
  return ORBFE_OK;
}

extern "C" int orbfe_matcher_last_stats(orbfe_matcher* m, int* rounds, int* serial_used) {
  if (!m) return ORBFE_ERR_ARG;
  if (rounds) *rounds = m->last_rounds;
  if (serial_used) *serial_used = m->last_serial;
  return ORBFE_OK;
}

// ---- isInFrustum / SearchLocalPoints ------------------------------------------------------------
static bool geom_ok(const orbfe_mappoint_geometry* g, bool need_desc) {
  return g && g->m >= 0 &&
         (g->m == 0 || (g->flags && g->world_pos && g->normal && g->min_distance && g->max_distance &&
                        (!need_desc || g->descriptors)));
}

static void fill_frustum_args(FrustumArgs& fa, const orbfe_frame_view* F, const float* T, float log_sf,
                              float cos_limit) {
  std::memset(&fa, 0, sizeof(fa));
  const float Rcw[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
  const float tcw[3] = {T[3], T[7], T[11]};
  std::memcpy(fa.rcw, Rcw, sizeof(Rcw));
  std::memcpy(fa.tcw, tcw, sizeof(tcw));
  for (int i = 0; i < 3; i++) {  // mOw = -mRcw.t() * mtcw (Frame.cc:314), double-accumulated
    double s = (double)Rcw[i] * (double)tcw[0];
    s += (double)Rcw[3 + i] * (double)tcw[1];
    s += (double)Rcw[6 + i] * (double)tcw[2];
    fa.ow[i] = -(float)s;
  }
  fa.fx = F->fx;
  fa.fy = F->fy;
  fa.cx = F->cx;
  fa.cy = F->cy;
  fa.bf = F->bf;
  fa.min_x = F->min_x;
  fa.max_x = F->max_x;
  fa.min_y = F->min_y;
  fa.max_y = F->max_y;
  fa.cos_limit = cos_limit;
  fa.nlevels = F->nlevels;
  predict_scale_table(log_sf, F->nlevels, fa.scale_thr);
}

struct FrustumPlan {
  size_t flags_in, pos, normal, mind, maxd, o_flags, o_px, o_py, o_pxr, o_lvl, o_vc, counter;
};
static FrustumPlan plan_frustum(Arena& ar, int M) {
  const size_t m1 = (size_t)std::max(M, 1);
  FrustumPlan p;
  p.flags_in = ar.add(m1);
  p.pos = ar.add(12 * m1);
  p.normal = ar.add(12 * m1);
  p.mind = ar.add(4 * m1);
  p.maxd = ar.add(4 * m1);
  p.o_flags = ar.add(m1);
  p.o_px = ar.add(4 * m1);
  p.o_py = ar.add(4 * m1);
  p.o_pxr = ar.add(4 * m1);
  p.o_lvl = ar.add(4 * m1);
  p.o_vc = ar.add(4 * m1);
  p.counter = ar.add(4);
  return p;
}
// stages the geometry, launches k_frustum; outputs stay in the arena
static int launch_frustum(orbfe_matcher* m, uint8_t* A, const FrustumPlan& p, const orbfe_mappoint_geometry* G,
                          FrustumArgs fa) {
  const size_t M = (size_t)G->m;
  stage_h2d(m, A + p.flags_in, G->flags, M);
  stage_h2d(m, A + p.pos, G->world_pos, 12 * M);
  stage_h2d(m, A + p.normal, G->normal, 12 * M);
  stage_h2d(m, A + p.mind, G->min_distance, 4 * M);
  stage_h2d(m, A + p.maxd, G->max_distance, 4 * M);
  int st = flush_h2d(m);
  if (st) return st;
  prof_begin(m);
  ORBFE_HIP_CHECK(hipMemsetAsync(A + p.counter, 0, 4, m->stream));
  fa.m = G->m;
  fa.flags_in = A + p.flags_in;
  fa.pos = (const float*)(A + p.pos);
  fa.normal = (const float*)(A + p.normal);
  fa.min_d = (const float*)(A + p.mind);
  fa.max_d = (const float*)(A + p.maxd);
  fa.out.flags = A + p.o_flags;
  fa.out.proj_x = (float*)(A + p.o_px);
  fa.out.proj_y = (float*)(A + p.o_py);
  fa.out.proj_xr = (float*)(A + p.o_pxr);
  fa.out.level = (int32_t*)(A + p.o_lvl);
  fa.out.view_cos = (float*)(A + p.o_vc);
  fa.n_in_view = (int32_t*)(A + p.counter);
  if (G->m > 0) ORBFE_LAUNCH("k_frustum", k_frustum, dim3((G->m + 255) / 256), dim3(256), 0, m->stream, fa);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}
// D2H of the per-MapPoint outputs the caller asked for, and the in-view count
static int fetch_frustum(orbfe_matcher* m, uint8_t* A, const FrustumPlan& p, int M, const orbfe_frustum_out* out,
                         int* n_in_view) {
  const size_t n = (size_t)M;
  if (out && M > 0) {
    if (out->flags) orbfe_mi::stage_d2h(m, out->flags, A + p.o_flags, n);
    if (out->proj_x) orbfe_mi::stage_d2h(m, out->proj_x, A + p.o_px, 4 * n);
    if (out->proj_y) orbfe_mi::stage_d2h(m, out->proj_y, A + p.o_py, 4 * n);
    if (out->proj_xr) orbfe_mi::stage_d2h(m, out->proj_xr, A + p.o_pxr, 4 * n);
    if (out->level) orbfe_mi::stage_d2h(m, out->level, A + p.o_lvl, 4 * n);
    if (out->view_cos) orbfe_mi::stage_d2h(m, out->view_cos, A + p.o_vc, 4 * n);
  }
  int32_t nv = 0;
  orbfe_mi::stage_d2h(m, &nv, A + p.counter, 4);
  const int st = orbfe_mi::fetch_d2h(m);
  if (st) return st;
  if (n_in_view) *n_in_view = nv;
  return ORBFE_OK;
}

extern "C" int orbfe_is_in_frustum(orbfe_matcher* m, const orbfe_frame_view* F, const orbfe_mappoint_geometry* G,
                                   const float* tcw, float log_scale_factor, float viewing_cos_limit,
                                   const orbfe_frustum_out* out, int* n_in_view) {
  if (!m || !F || !tcw || !geom_ok(G, false) || F->nlevels <= 0 || F->nlevels > ORBFE_MAX_LEVELS_M)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_is_in_frustum: bad argument");
  hipSetDevice(m->device);
  Arena ar;
  const FrustumPlan p = plan_frustum(ar, G->m);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  FrustumArgs fa;
  fill_frustum_args(fa, F, tcw, log_scale_factor, viewing_cos_limit);
  m->prof_started = m->prof_done = false;  // this call's own device-time window (k_frustum)
  if ((st = launch_frustum(m, m->arena, p, G, fa))) return st;
  prof_end(m);
  return fetch_frustum(m, m->arena, p, G->m, out, n_in_view);
}

extern "C" int orbfe_search_local_points(orbfe_matcher* m, const orbfe_frame_view* F,
                                         const orbfe_mappoint_geometry* G, const float* tcw,
                                         float log_scale_factor, float viewing_cos_limit, float th,
                                         int32_t* best_idx, int* nmatches, const orbfe_frustum_out* out,
                                         int* n_in_view) {
  if (!m || !frame_ok(F) || !tcw || !geom_ok(G, true) || !nmatches || (G->m > 0 && !best_idx))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_local_points: bad argument");
  hipSetDevice(m->device);
  const int M = G->m;
  FrustumPlan fp;
  FrustumArgs fa;
  fill_frustum_args(fa, F, tcw, log_scale_factor, viewing_cos_limit);
  uint8_t* A_used = nullptr;
  auto plan = [&](Arena& ar) -> int {
    fp = plan_frustum(ar, M);
    return 0;
  };
  auto make = [&](uint8_t* A, const orbfe_frame_view& dF, SbpQuery* dq) -> int {
    A_used = A;
    int st = launch_frustum(m, A, fp, G, fa);
    if (st) return st;
    // SearchByProjection's queries straight from the isInFrustum outputs (no host round trip);
    // with nothing in view every query is empty and the result is the skipped matcher's
    LocalQueryArgs qa;
    std::memset(&qa, 0, sizeof(qa));
    qa.mp.m = M;
    qa.mp.flags = A + fp.o_flags;
    qa.mp.proj_x = (const float*)(A + fp.o_px);
    qa.mp.proj_y = (const float*)(A + fp.o_py);
    qa.mp.proj_xr = (const float*)(A + fp.o_pxr);
    qa.mp.level = (const int32_t*)(A + fp.o_lvl);
    qa.mp.view_cos = (const float*)(A + fp.o_vc);
    qa.scale_factors = dF.scale_factors;
    qa.th = th;
    qa.q = dq;
    ORBFE_LAUNCH("k_sbp_local_queries", k_sbp_local_queries, dim3((M + 255) / 256), dim3(256), 0, m->stream, qa);
    return ORBFE_OK;
  };
  int st = run_sbp(m, F, M, SbpMode{0, TH_HIGH, 0, 0}, G->descriptors, nullptr, plan, make, best_idx, nmatches);
  if (st) return st;
  if (M == 0) {
    if (n_in_view) *n_in_view = 0;
    return ORBFE_OK;
  }
  return fetch_frustum(m, A_used, fp, M, out, n_in_view);
}
