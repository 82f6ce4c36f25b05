// orbfe_bow.hip -- SearchByBoW (both overloads), SearchForInitialization and
// MapPoint::ComputeDistinctiveDescriptors on CDNA4 (gfx950, wave64).
//
// Reference: lreithmayr/ORB_SLAM2_2021.
//   SearchByBoW(KeyFrame*, Frame&, ..)   src/ORBmatcher.cc:165-293
//   SearchByBoW(KeyFrame*, KeyFrame*, ..) src/ORBmatcher.cc:536-669
//     Keypoints only meet inside one vocabulary node and each keypoint sits in exactly one node,
//     so nodes are independent: one wavefront per common node. The node's candidates (Frame /
//     KF2 side) are spread over the lanes with their descriptors in LDS; the KF features are
//     walked in order (the claim order of vpMapPointMatches / vbMatched2), each step one pass of
//     distances plus two wave reductions: the first minimum (distance, then position) and the
//     second-smallest distance of the multiset -- exactly bestDist1 / bestIdx / bestDist2 of the
//     reference loop. k_bow_finish applies the rotation-consistency filter per pair.
//   SearchForInitialization  src/ORBmatcher.cc:414-534
//     The window gather + distances run on the projection engine's round 0 (16 lanes per query,
//     candidate cache sized to hold every level-0 keypoint); the order-dependent part (a later
//     feature can take a keypoint from an earlier one when it is closer) is one wavefront walking
//     the features in order over the cached (keypoint, distance) lists, with vMatchedDistance and
//     vnMatches21 in LDS.
//   MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:272-337
//     One wavefront per MapPoint: row i of the distance matrix across the lanes, its median by a
//     9-step bisection on the distance value with ballot counts, first minimum over rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_keyframe.h"
#include "orbfe_device.h"
#include "orbfe_match_internal.h"
#include "orbfe_ktimer.h"

using namespace orbfe_mi;

#define BOW_LDS_CAND 128  // node candidates whose descriptors sit in LDS (larger nodes read L2)
#define BOW_MAX_NODE SFT_MAX_KF2
#define DD_MAX_OBS 4096   // observations per MapPoint in ComputeDistinctiveDescriptors

namespace {
struct BowPair {
  orbfe_frame_view A, B;       // A: the KeyFrame walked in order; B: candidates (Frame / KF2)
  orbfe_feature_vector fa, fb;
  int32_t* match_a;            // per A keypoint: B keypoint or -1
  int32_t* out_b;              // mode 0: per B keypoint, the A keypoint assigned to it, or -1
  int32_t* nmatches;
  int mode;                    // 0 KeyFrame -> Frame (:165-293), 1 KeyFrame -> KeyFrame (:536-669)
};

__device__ __forceinline__ bool good_mp(uint8_t st) { return st != ORBFE_MP_NONE && st != ORBFE_MP_BAD; }

__global__ __launch_bounds__(256) void k_bow_init(const BowPair* pairs) {
  const BowPair P = pairs[blockIdx.x];  // a private copy: stores through P.match_a cannot alias it
  for (int i = threadIdx.x; i < P.A.n; i += 256) P.match_a[i] = -1;
  if (P.out_b)
    for (int i = threadIdx.x; i < P.B.n; i += 256) P.out_b[i] = -1;
}

__global__ __launch_bounds__(256) void k_bow_nodes(const BowPair* pairs, float nnratio) {
  __shared__ uint4 s_desc[4][BOW_LDS_CAND * 2];
  __shared__ uint32_t s_taken[4][BOW_MAX_NODE / 32];  // unusable or claimed candidates
  const BowPair P = pairs[blockIdx.y];
  const int w = wave_id(), lane = lane_id();
  const int a = blockIdx.x * 4 + w;
  if (a >= P.fa.n_nodes) return;
  const uint32_t id = P.fa.node_ids[a];
  const int o1 = P.fa.offsets[a], e1 = P.fa.offsets[a + 1];
  // the merge-join visits exactly the common node ids (:186-270): find id among B's node ids
  int lo = -1;
  for (int b = 0; b < P.fb.n_nodes && lo < 0; b += 128) {
    const int i0 = b + lane, i1 = b + 64 + lane;
    const uint32_t v0 = i0 < P.fb.n_nodes ? P.fb.node_ids[i0] : ~0u;
    const uint32_t v1 = i1 < P.fb.n_nodes ? P.fb.node_ids[i1] : ~0u;
    const uint64_t m0 = wave_ballot(v0 == id), m1 = wave_ballot(v1 == id);
    if (m0) lo = b + __builtin_ctzll(m0);
    else if (m1) lo = b + 64 + __builtin_ctzll(m1);
  }
  if (lo < 0) return;
  const int o2 = P.fb.offsets[lo], n2 = P.fb.offsets[lo + 1] - o2;
  if (n2 > BOW_MAX_NODE) return;  // rejected on the host
  uint4* cd = s_desc[w];
  uint32_t* taken = s_taken[w];
  // candidates: descriptors of the first BOW_LDS_CAND in LDS; "taken" starts as "unusable"
  // (mode 1: no MapPoint or a bad one, :590-594)
  for (int wd = lane; wd < (n2 + 31) / 32; wd += 64) {
    uint32_t bits = 0;
    for (int k = 0; k < 32; k++) {
      const int p = 32 * wd + k;
      if (p < n2 && P.mode == 1 && !good_mp(P.B.mp_state[P.fb.indices[o2 + p]])) bits |= 1u << k;
    }
    taken[wd] = bits;
  }
  for (int p = lane; p < min(n2, BOW_LDS_CAND); p += 64) {
    const int idx2 = P.fb.indices[o2 + p];
    load_desc(P.B.descriptors + (size_t)idx2 * 32, cd[2 * p], cd[2 * p + 1]);
  }
  wave_sync();
  const unsigned NONE = (256u << 16) | 0xffffu;
  for (int b1 = o1; b1 < e1; b1 += 64) {
    // 64 A features at a time, one per lane; the walk below broadcasts them with readlane
    const int my = b1 + lane;
    int m_idx = -1;
    bool m_ok = false;
    uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
    if (my < e1) {
      m_idx = P.fa.indices[my];
      m_ok = good_mp(P.A.mp_state[m_idx]);  // !pMP || isBad (:199-203, :572-576)
      if (m_ok) load_desc(P.A.descriptors + (size_t)m_idx * 32, m0, m1);
    }
    const uint64_t okmask = wave_ballot(m_ok);
    const int nb = min(64, e1 - b1);
    for (int q = 0; q < nb; q++) {
      if (!((okmask >> q) & 1ull)) continue;
      uint4 a0, a1;
      a0.x = __builtin_amdgcn_readlane(m0.x, q);
      a0.y = __builtin_amdgcn_readlane(m0.y, q);
      a0.z = __builtin_amdgcn_readlane(m0.z, q);
      a0.w = __builtin_amdgcn_readlane(m0.w, q);
      a1.x = __builtin_amdgcn_readlane(m1.x, q);
      a1.y = __builtin_amdgcn_readlane(m1.y, q);
      a1.z = __builtin_amdgcn_readlane(m1.z, q);
      a1.w = __builtin_amdgcn_readlane(m1.w, q);
      // lane-local first minimum (distance << 16 | position) and second-smallest distance
      unsigned k1 = NONE;
      int d2 = 256;
      for (int p = lane; p < n2; p += 64) {
        if ((taken[p >> 5] >> (p & 31)) & 1u) continue;
        uint4 c0, c1;
        if (p < BOW_LDS_CAND) {
          c0 = cd[2 * p];
          c1 = cd[2 * p + 1];
        } else {
          load_desc(P.B.descriptors + (size_t)P.fb.indices[o2 + p] * 32, c0, c1);
        }
        const int d = hamming256(a0, a1, c0, c1);
        const unsigned key = ((unsigned)d << 16) | (unsigned)p;
        if (key < k1) {
          d2 = min(d2, (int)(k1 >> 16));
          k1 = key;
        } else if (d < d2) {
          d2 = d;
        }
      }
      const unsigned kmin = (unsigned)wave_min((int)k1);
      const int second = wave_min(k1 == kmin ? d2 : (int)(k1 >> 16));
      const int bestDist1 = (int)(kmin >> 16);
      const bool acc = (P.mode == 0 ? bestDist1 <= TH_LOW : bestDist1 < TH_LOW) &&
                       (float)bestDist1 < nnratio * (float)second;  // :234-236, :612-614
      if (acc) {
        const int p = (int)(kmin & 0xffffu);
        if (lane == 0) {
          taken[p >> 5] |= 1u << (p & 31);  // vpMapPointMatches[bestIdxF] / vbMatched2[bestIdx2]
          P.match_a[__builtin_amdgcn_readlane(m_idx, q)] = P.fb.indices[o2 + p];
        }
        wave_sync();
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_bow_finish(const BowPair* pairs, int check_ori) {
  __shared__ int s_hist[HISTO_LENGTH];
  __shared__ int s_misc[8];
  const BowPair P = pairs[blockIdx.x];  // a private copy: stores through P.match_a cannot alias it
  const int t = threadIdx.x;
  if (t < HISTO_LENGTH) s_hist[t] = 0;
  if (t == 0) s_misc[4] = 0;
  __syncthreads();
  if (check_ori) {  // :272-290, :648-666
    for (int i = t; i < P.A.n; i += 256) {
      const int b = P.match_a[i];
      if (b >= 0) atomicAdd(&s_hist[rot_bin_dev(P.A.keys_un[i].angle, P.B.keys_un[b].angle)], 1);
    }
    __syncthreads();
    if (t == 0) three_maxima_dev(s_hist, s_misc[0], s_misc[1], s_misc[2]);
    __syncthreads();
  }
  int cnt = 0;
  for (int i = t; i < P.A.n; i += 256) {
    const int b = P.match_a[i];
    if (b < 0) continue;
    if (check_ori) {
      const int bin = rot_bin_dev(P.A.keys_un[i].angle, P.B.keys_un[b].angle);
      if (bin != s_misc[0] && bin != s_misc[1] && bin != s_misc[2]) {
        P.match_a[i] = -1;
        continue;
      }
    }
    if (P.out_b) P.out_b[b] = i;
    cnt++;
  }
  cnt = wave_sum(cnt);
  if (lane_id() == 0) atomicAdd(&s_misc[4], cnt);
  __syncthreads();
  if (t == 0) *P.nmatches = s_misc[4];
}

// ---- SearchForInitialization ----------------------------------------------------------------------
// The order dependence of :431-501 as a fixpoint (k_init_round). Feature i1's decision D(i1) -- the
// accepted bestIdx2, or none -- depends only on vMatchedDistance as the features before it left it,
// and vMatchedDistance[i2] is then the smallest accepted distance among the earlier features that
// chose i2 (an assignment needs a strictly smaller distance, :458). Round r recomputes every
// decision against the choosers of round r-1 (per i2 up to INIT_SLOTS (i1, dist) entries); two equal
// consecutive rounds with complete chooser lists are the sequential result (D(i) = f(D(j < i)) has a
// single solution, and round r has the first r features right). Otherwise k_init_seq walks the
// features in order.
#define INIT_SLOTS 16
#define INIT_MAX_ROUNDS 16
#define INIT_STATE_INTS (2 + 2 * INIT_MAX_ROUNDS)  // settled, rounds run, changed[r], overflow[r]
#define INIT_CHANGED(r) (2 + (r))
#define INIT_OVF(r) (2 + INIT_MAX_ROUNDS + (r))

struct InitQueryArgs {
  int n1, n2;
  const orbfe_keypoint* keys1;
  const float* prev;
  float r;
  SbpQuery* q;
  int32_t* dec_init;  // round 0's "previous" decisions: never computed
  int32_t* cnt0;      // chooser counts written by round 0 and read as round -1's: zero
  int32_t* cnt2;
  int32_t* state;
};
__global__ __launch_bounds__(256) void k_init_queries(InitQueryArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.n2) {
    a.cnt0[i] = 0;
    a.cnt2[i] = 0;
  }
  if (i < INIT_STATE_INTS) a.state[i] = 0;
  if (i >= a.n1) return;
  a.dec_init[i] = (int32_t)0xfefefefe;
  SbpQuery q = {};
  q.gate = SBP_GATE_NONE;
  const int level1 = a.keys1[i].octave;
  if (level1 <= 0) {  // level1 > 0: continue (:435-436); window at level1..level1 (:438-439)
    q.x = a.prev[2 * i];
    q.y = a.prev[2 * i + 1];
    q.r = a.r;
    q.min_level = level1;
    q.max_level = level1;
    q.flags = 1;
  }
  a.q[i] = q;
}

struct InitFixArgs {
  int n1, n2, cand_cap, round;
  float nnratio;
  const uint32_t* cand;  // SearchByProjection's candidate cache: keypoint | distance << 16 | level << 24
  const int32_t* cand_n;
  const int32_t* dec_prev;
  int32_t* dec_cur;          // accepted i2, or -1
  const int2* slots_prev;    // choosers of round r-1: per i2, INIT_SLOTS (i1, dist)
  const int32_t* cnt_prev;
  int2* slots_cur;
  int32_t* cnt_cur;
  int32_t* cnt_next;         // cleared here for round r+1
  int32_t* state;
};

// after `rounds` rounds: the last reproduced the one before it, and neither chooser list overflowed
__device__ __forceinline__ bool init_settled(const int32_t* st, int rounds) {
  return rounds >= 2 && st[INIT_CHANGED(rounds - 1)] == 0 && st[INIT_OVF(rounds - 1)] == 0 &&
         st[INIT_OVF(rounds - 2)] == 0;
}

__global__ __launch_bounds__(256) void k_init_round(InitFixArgs a) {
  if (a.state[0] != 0 || init_settled(a.state, a.round)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.state[0] = 1;
    return;
  }
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t == 0) a.state[1] = a.round + 1;
  if (t < a.n2) a.cnt_next[t] = 0;
  const int j = threadIdx.x & 15, row = threadIdx.x >> 4;
  const int i1 = blockIdx.x * 16 + row;
  if (i1 >= a.n1) return;  // the 16 lanes of a row leave together
  const int n = a.cand_n[i1];
  const uint32_t* ce = a.cand + (size_t)i1 * a.cand_cap;
  const unsigned NONE = 0xffffffffu;
  unsigned k1 = NONE;  // (distance << 16 | position)
  int d2 = INT_MAX;
  for (int c = j; c < n; c += 16) {
    const uint32_t e = ce[c];
    const int i2 = cand_key(e);
    const int dist = cand_dist(e);
    int vmd = INT_MAX;  // vMatchedDistance[i2] before i1, per the previous round's choosers
    const int cc = min(a.cnt_prev[i2], INIT_SLOTS);
    for (int s = 0; s < cc; s++) {
      const int2 e = a.slots_prev[(size_t)i2 * INIT_SLOTS + s];
      if (e.x < i1) vmd = min(vmd, e.y);
    }
    if (vmd <= dist) continue;  // :458-459
    const unsigned key = ((unsigned)dist << 16) | (unsigned)c;
    if (key < k1) {
      if (k1 != NONE) d2 = min(d2, (int)(k1 >> 16));
      k1 = key;
    } else if (dist < d2) {
      d2 = dist;
    }
  }
  unsigned kmin = k1;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    const unsigned other = (unsigned)__shfl_xor((int)kmin, o, 16);
    kmin = other < kmin ? other : kmin;
  }
  int second = k1 == kmin ? d2 : (k1 == NONE ? INT_MAX : (int)(k1 >> 16));
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) second = min(second, __shfl_xor(second, o, 16));
  int dec = -1;
  if (kmin != NONE) {
    const int bestDist = (int)(kmin >> 16);
    if (bestDist <= TH_LOW && (float)bestDist < (float)second * a.nnratio) dec = cand_key(ce[kmin & 0xffffu]);  // :473-475
  }
  bool changed = false;
  if (j == 0) {
    a.dec_cur[i1] = dec;
    changed = dec != a.dec_prev[i1];
    if (dec >= 0) {
      const int s = atomicAdd(&a.cnt_cur[dec], 1);
      if (s < INIT_SLOTS) a.slots_cur[(size_t)dec * INIT_SLOTS + s] = make_int2(i1, (int)(kmin >> 16));
      else a.state[INIT_OVF(a.round)] = 1;
    }
  }
  if (wave_ballot(changed) && lane_id() == __ffsll((long long)wave_ballot(true)) - 1)
    a.state[INIT_CHANGED(a.round)] = 1;  // plain store: every writer stores 1
}

struct InitSeqArgs {
  int n1, n2, cand_cap, check_ori;
  float nnratio;
  const uint32_t* cand;
  const int32_t* cand_n;
  const orbfe_keypoint* keys1;
  const orbfe_keypoint* keys2;
  int32_t* match12;
  int32_t* bin_of;   // rotation bin of every feature pushed into rotHist, else -1
  float* prev;
  int32_t* nmatches;
  // the fixpoint's outcome: decisions by round parity, choosers by round mod 3
  const int32_t* state;
  const int32_t* dec[2];
  const int2* slots[3];
  const int32_t* cnt[3];
};

// One wavefront: the fixpoint's result when it settled (the last accepted chooser of an i2 keeps
// it, :477-481; every accepted feature was pushed into rotHist, :496), else the reference's loop
// over i1 in order (:431-501); then the rotation filter (:503-526) and the vbPrevMatched update
// (:528-531).
__global__ __launch_bounds__(64) void k_init_seq(InitSeqArgs a) {
  extern __shared__ int s_init[];  // vMatchedDistance[n2], vnMatches21[n2], hist[30], misc[4]
  int* mdist = s_init;
  int* m21 = s_init + a.n2;
  int* hist = m21 + a.n2;
  int* misc = hist + HISTO_LENGTH;
  const int lane = lane_id();
  if (lane < HISTO_LENGTH) hist[lane] = 0;
  const int rounds = a.state[1];
  const bool settled = a.state[0] != 0 || init_settled(a.state, rounds);
  if (settled) {
    const int32_t* D = a.dec[(rounds - 1) & 1];
    const int2* S = a.slots[(rounds - 1) % 3];
    const int32_t* C = a.cnt[(rounds - 1) % 3];
    for (int i = lane; i < a.n1; i += 64) {
      const int d = D[i];
      int last = -1;  // the last feature that chose d keeps it
      if (d >= 0)
        for (int s = 0; s < C[d]; s++) last = max(last, S[(size_t)d * INIT_SLOTS + s].x);
      a.match12[i] = (d >= 0 && last == i) ? d : -1;
      a.bin_of[i] = (d >= 0 && a.check_ori) ? rot_bin_dev(a.keys1[i].angle, a.keys2[d].angle) : -1;
    }
  } else {
    for (int k = lane; k < a.n2; k += 64) {
      mdist[k] = INT_MAX;
      m21[k] = -1;
    }
    for (int i = lane; i < a.n1; i += 64) {
      a.match12[i] = -1;
      a.bin_of[i] = -1;
    }
  }
  wave_sync();
  const unsigned NONE = 0xffffffffu;
  for (int i1 = 0; i1 < a.n1 && !settled; i1++) {
    const int n = a.cand_n[i1];
    if (n <= 0) continue;  // not level 0, or vIndices2.empty()
    const uint32_t* ce = a.cand + (size_t)i1 * a.cand_cap;
    unsigned k1 = NONE;  // (distance << 16 | position)
    int d2 = INT_MAX;
    for (int j = lane; j < n; j += 64) {
      const uint32_t e = ce[j];
      const int i2 = cand_key(e);
      const int dist = cand_dist(e);
      if (mdist[i2] <= dist) continue;  // vMatchedDistance[i2] <= dist (:458-459)
      const unsigned key = ((unsigned)dist << 16) | (unsigned)j;
      if (key < k1) {
        if (k1 != NONE) d2 = min(d2, (int)(k1 >> 16));
        k1 = key;
      } else if (dist < d2) {
        d2 = dist;
      }
    }
    const unsigned kmin = (unsigned)wave_min((int)(k1 ^ 0x80000000u)) ^ 0x80000000u;  // unsigned min
    const int lane_second = k1 == kmin ? d2 : (k1 == NONE ? INT_MAX : (int)(k1 >> 16));
    const int bestDist2 = wave_min(lane_second);
    if (kmin == NONE) continue;
    const int bestDist = (int)(kmin >> 16);
    if (bestDist <= TH_LOW && (float)bestDist < (float)bestDist2 * a.nnratio) {  // :473-475
      const int bestIdx2 = cand_key(ce[kmin & 0xffffu]);
      if (lane == 0) {
        const int prev1 = m21[bestIdx2];
        if (prev1 >= 0) a.match12[prev1] = -1;  // :477-481
        a.match12[i1] = bestIdx2;
        m21[bestIdx2] = i1;
        mdist[bestIdx2] = bestDist;
        if (a.check_ori) a.bin_of[i1] = rot_bin_dev(a.keys1[i1].angle, a.keys2[bestIdx2].angle);
      }
      wave_sync();
    }
  }
  __threadfence_block();
  wave_sync();
  if (a.check_ori) {
    for (int i = lane; i < a.n1; i += 64) {
      const int b = a.bin_of[i];
      if (b >= 0) atomicAdd(&hist[b], 1);
    }
    wave_sync();
    if (lane == 0) three_maxima_dev(hist, misc[0], misc[1], misc[2]);
    wave_sync();
    for (int i = lane; i < a.n1; i += 64) {
      const int b = a.bin_of[i];
      if (b >= 0 && b != misc[0] && b != misc[1] && b != misc[2]) a.match12[i] = -1;
    }
  }
  int cnt = 0;
  for (int i = lane; i < a.n1; i += 64) {
    const int m = a.match12[i];
    if (m >= 0) {
      cnt++;
      a.prev[2 * i] = a.keys2[m].x;
      a.prev[2 * i + 1] = a.keys2[m].y;
    }
  }
  cnt = wave_sum(cnt);
  if (lane == 0) *a.nmatches = cnt;
}

// ---- ComputeDistinctiveDescriptors --------------------------------------------------------------
__global__ __launch_bounds__(256) void k_distinctive(int n_points, const int32_t* offsets, const uint8_t* desc,
                                                     int32_t* best_index) {
  __shared__ uint16_t s_row[4][DD_MAX_OBS];
  const int w = wave_id(), lane = lane_id();
  const int pt = blockIdx.x * 4 + w;
  if (pt >= n_points) return;
  const int o = offsets[pt];
  const int N = offsets[pt + 1] - o;
  if (N <= 0 || N > DD_MAX_OBS) {
    if (lane == 0) best_index[pt] = -1;  // vDescriptors.empty(): return (:299-300)
    return;
  }
  const int kth = (N - 1) >> 1;  // vDists[0.5 * (N - 1)] (:324)
  uint16_t* row = s_row[w];
  int bestMedian = INT_MAX, bestIdx = 0;
  uint4 mine0 = make_uint4(0, 0, 0, 0), mine1 = mine0;
  if (lane < N) load_desc(desc + 32 * (size_t)(o + lane), mine0, mine1);
  for (int i = 0; i < N; i++) {
    uint4 q0, q1;
    if (i < 64) {  // row i's descriptor from its lane
      q0.x = __builtin_amdgcn_readlane(mine0.x, i);
      q0.y = __builtin_amdgcn_readlane(mine0.y, i);
      q0.z = __builtin_amdgcn_readlane(mine0.z, i);
      q0.w = __builtin_amdgcn_readlane(mine0.w, i);
      q1.x = __builtin_amdgcn_readlane(mine1.x, i);
      q1.y = __builtin_amdgcn_readlane(mine1.y, i);
      q1.z = __builtin_amdgcn_readlane(mine1.z, i);
      q1.w = __builtin_amdgcn_readlane(mine1.w, i);
    } else {
      load_desc(desc + 32 * (size_t)(o + i), q0, q1);
    }
    int median;
    if (N <= 64) {
      const int d = lane < N ? (lane == i ? 0 : hamming256(q0, q1, mine0, mine1)) : 512;
      int lo = 0, hi = 256;  // smallest t with #{d <= t} > kth
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__popcll(wave_ballot(d <= mid)) > kth) hi = mid;
        else lo = mid + 1;
      }
      median = lo;
    } else {
      for (int j = lane; j < N; j += 64) {
        uint4 c0, c1;
        if (j < 64) {
          c0 = mine0;
          c1 = mine1;
        } else {
          load_desc(desc + 32 * (size_t)(o + j), c0, c1);
        }
        row[j] = (uint16_t)(j == i ? 0 : hamming256(q0, q1, c0, c1));
      }
      wave_sync();
      int lo = 0, hi = 256;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int c = 0;
        for (int j = lane; j < N; j += 64) c += row[j] <= mid;
        if (wave_sum(c) > kth) hi = mid;
        else lo = mid + 1;
      }
      median = lo;
      wave_sync();
    }
    if (median < bestMedian) {  // first minimum (:326-330)
      bestMedian = median;
      bestIdx = i;
    }
  }
  if (lane == 0) best_index[pt] = bestIdx;
}

// ---- host -----------------------------------------------------------------------------------------
struct FvOffsets {
  size_t ids, offs, idx;
};
FvOffsets plan_fv(Arena& ar, const orbfe_feature_vector* fv) {
  FvOffsets o;
  o.ids = ar.add(4 * (size_t)std::max(fv->n_nodes, 1));
  o.offs = ar.add(4 * (size_t)(fv->n_nodes + 1));
  o.idx = ar.add(4 * (size_t)std::max(fv->n_nodes > 0 ? fv->offsets[fv->n_nodes] : 0, 1));
  return o;
}
void upload_fv(orbfe_matcher* m, const FvOffsets& o, const orbfe_feature_vector* fv, orbfe_feature_vector* d) {
  uint8_t* A = m->arena;
  d->n_nodes = fv->n_nodes;
  d->node_ids = (const uint32_t*)(A + o.ids);
  d->offsets = (const int32_t*)(A + o.offs);
  d->indices = (const int32_t*)(A + o.idx);
  if (fv->n_nodes > 0) {
    const int ni = fv->offsets[fv->n_nodes];
    stage_h2d(m, A + o.ids, fv->node_ids, 4 * (size_t)fv->n_nodes);
    stage_h2d(m, A + o.offs, fv->offsets, 4 * (size_t)(fv->n_nodes + 1));
    if (ni > 0) stage_h2d(m, A + o.idx, fv->indices, 4 * (size_t)ni);
  } else {
    const int32_t zero = 0;
    stage_h2d(m, A + o.offs, &zero, 4);
  }
}
bool fv_ok(const orbfe_feature_vector* fv, int n) {
  if (!fv || fv->n_nodes < 0) return false;
  if (fv->n_nodes == 0) return true;
  if (!fv->node_ids || !fv->offsets || !fv->indices || fv->offsets[0] != 0) return false;
  for (int k = 0; k < fv->n_nodes; k++) {
    if (fv->offsets[k + 1] < fv->offsets[k]) return false;
    if (fv->offsets[k + 1] - fv->offsets[k] > BOW_MAX_NODE) return false;
    if (k > 0 && fv->node_ids[k] <= fv->node_ids[k - 1]) return false;
  }
  for (int j = 0; j < fv->offsets[fv->n_nodes]; j++)
    if (fv->indices[j] < 0 || fv->indices[j] >= n) return false;
  return true;
}

// n_a KeyFrames (A side) against B; B is a shared Frame (mode 0) or one KF2 per pair (mode 1).
int run_bow(orbfe_matcher* m, int mode, int n_pairs, const orbfe_frame_view* As, const orbfe_feature_vector* fas,
            const orbfe_frame_view* Bs, const orbfe_feature_vector* fbs, bool shared_b, int32_t* out, int32_t* counts) {
  hipSetDevice(m->device);
  Arena ar;
  std::vector<FrameOffsets> oa(n_pairs), ob(shared_b ? 1 : n_pairs);
  std::vector<FvOffsets> fa(n_pairs), fb(shared_b ? 1 : n_pairs);
  for (int p = 0; p < n_pairs; p++) {
    oa[p] = plan_frame(ar, &As[p]);
    fa[p] = plan_fv(ar, &fas[p]);
  }
  for (size_t p = 0; p < ob.size(); p++) {
    ob[p] = plan_frame(ar, &Bs[p]);
    fb[p] = plan_fv(ar, &fbs[p]);
  }
  const size_t opairs = ar.add(sizeof(BowPair) * n_pairs);
  std::vector<size_t> omatch(n_pairs), oout(n_pairs);
  for (int p = 0; p < n_pairs; p++) {
    omatch[p] = ar.add(4 * (size_t)std::max(As[p].n, 1));
    oout[p] = ar.add(mode == 0 ? 4 * (size_t)std::max(Bs[shared_b ? 0 : p].n, 1) : 0);
  }
  const size_t ocounts = ar.add(4 * (size_t)n_pairs);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  uint8_t* A = m->arena;
  std::vector<orbfe_frame_view> dB(ob.size());
  std::vector<orbfe_feature_vector> dfb(ob.size());
  for (size_t p = 0; p < ob.size(); p++) {
    if ((st = upload_frame(m, ob[p], &Bs[p], &dB[p]))) return st;
    upload_fv(m, fb[p], &fbs[p], &dfb[p]);
  }
  std::vector<BowPair> pairs(n_pairs);
  int max_nodes = 1;
  for (int p = 0; p < n_pairs; p++) {
    BowPair& P = pairs[p];
    std::memset(&P, 0, sizeof(P));
    if ((st = upload_frame(m, oa[p], &As[p], &P.A))) return st;
    upload_fv(m, fa[p], &fas[p], &P.fa);
    P.B = dB[shared_b ? 0 : p];
    P.fb = dfb[shared_b ? 0 : p];
    P.match_a = (int32_t*)(A + omatch[p]);
    P.out_b = mode == 0 ? (int32_t*)(A + oout[p]) : nullptr;
    P.nmatches = (int32_t*)(A + ocounts) + p;
    P.mode = mode;
    max_nodes = std::max(max_nodes, fas[p].n_nodes);
  }
  stage_h2d(m, A + opairs, pairs.data(), sizeof(BowPair) * n_pairs);
  if ((st = flush_h2d(m))) return st;
  const BowPair* dp = (const BowPair*)(A + opairs);
  ORBFE_LAUNCH("k_bow_init", k_bow_init, dim3(n_pairs), dim3(256), 0, m->stream, dp);
  ORBFE_LAUNCH("k_bow_nodes", k_bow_nodes, dim3((max_nodes + 3) / 4, n_pairs), dim3(256), 0, m->stream, dp, m->nnratio);
  ORBFE_LAUNCH("k_bow_finish", k_bow_finish, dim3(n_pairs), dim3(256), 0, m->stream, dp, m->check_ori);
  ORBFE_HIP_CHECK(hipGetLastError());
  size_t off = 0;
  for (int p = 0; p < n_pairs; p++) {  // mode 0: per Frame keypoint; mode 1: per KF1 keypoint
    const int n = mode == 0 ? Bs[shared_b ? 0 : p].n : As[p].n;
    if (n > 0) orbfe_mi::stage_d2h(m, out + off, A + (mode == 0 ? oout[p] : omatch[p]), 4 * (size_t)n);
    off += (size_t)n;
  }
  orbfe_mi::stage_d2h(m, counts, A + ocounts, 4 * (size_t)n_pairs);
  return orbfe_mi::fetch_d2h(m);
}

bool bow_frame_ok(const orbfe_frame_view* f) {
  return f && f->n >= 0 && f->n <= BOW_MAX_NODE * 4 && (f->n == 0 || (f->keys_un && f->descriptors && f->mp_state)) &&
         f->nlevels > 0 && f->scale_factors;
}
}  // namespace

extern "C" int orbfe_search_by_bow_kf_frame_multi(orbfe_matcher* m, int n_kf, const orbfe_frame_view* kfs,
                                                  const orbfe_feature_vector* kf_fvs, const orbfe_frame_view* frame,
                                                  const orbfe_feature_vector* frame_fv, int32_t* match_f,
                                                  int32_t* nmatches) {
  if (!m || n_kf < 0 || (n_kf > 0 && (!kfs || !kf_fvs || !nmatches)) || !bow_frame_ok(frame) ||
      !fv_ok(frame_fv, frame->n) || (n_kf > 0 && frame->n > 0 && !match_f))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_bow_kf_frame: bad argument");
  for (int i = 0; i < n_kf; i++)
    if (!bow_frame_ok(&kfs[i]) || !fv_ok(&kf_fvs[i], kfs[i].n))
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_bow_kf_frame: bad KeyFrame or FeatureVector");
  if (n_kf == 0) return ORBFE_OK;
  return run_bow(m, 0, n_kf, kfs, kf_fvs, frame, frame_fv, true, match_f, nmatches);
}

extern "C" int orbfe_search_by_bow_kf_frame(orbfe_matcher* m, const orbfe_frame_view* kf,
                                            const orbfe_feature_vector* kf_fv, const orbfe_frame_view* frame,
                                            const orbfe_feature_vector* frame_fv, int32_t* match_f, int* nmatches) {
  if (!nmatches) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_bow_kf_frame: nmatches is NULL");
  int32_t n = 0;
  const int st = orbfe_search_by_bow_kf_frame_multi(m, 1, kf, kf_fv, frame, frame_fv, match_f, &n);
  *nmatches = n;
  return st;
}

extern "C" int orbfe_search_by_bow_kf_kf(orbfe_matcher* m, const orbfe_frame_view* kf1,
                                         const orbfe_feature_vector* fv1, const orbfe_frame_view* kf2,
                                         const orbfe_feature_vector* fv2, int32_t* match12, int* nmatches) {
  if (!m || !bow_frame_ok(kf1) || !bow_frame_ok(kf2) || !fv_ok(fv1, kf1->n) || !fv_ok(fv2, kf2->n) || !nmatches ||
      (kf1->n > 0 && !match12))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_bow_kf_kf: bad argument");
  int32_t n = 0;
  const int st = run_bow(m, 1, 1, kf1, fv1, kf2, fv2, false, match12, &n);
  *nmatches = n;
  return st;
}

extern "C" int orbfe_search_for_initialization(orbfe_matcher* m, const orbfe_frame_view* f1,
                                               const orbfe_frame_view* f2, float* prev_matched, int window_size,
                                               int32_t* match12, int* nmatches) {
  if (!m || !frame_ok(f1) || !frame_ok(f2) || !nmatches || (f1->n > 0 && (!prev_matched || !match12)) ||
      f2->n > 32767)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_for_initialization: bad argument");
  if (f1->n == 0) {
    *nmatches = 0;
    return ORBFE_OK;
  }
  hipSetDevice(m->device);
  // every candidate is a level-0 keypoint of F2 (the window is level1..level1 = 0..0), so a cache
  // as large as that set never overflows
  int cap = 1;
  for (int k = 0; k < f2->n; k++) cap += f2->keys_un[k].octave == 0;
  const int n1 = f1->n, n2 = f2->n;
  const size_t n2s = (size_t)std::max(n2, 1);
  Arena ar;
  SbpPlan p;
  sbp_plan_inputs(ar, f2, n1, cap, p);
  const FrameOffsets o1 = plan_frame(ar, f1);
  const size_t oprev = ar.add(8 * (size_t)n1);
  sbp_plan_scratch(ar, f2, p);
  const size_t om = ar.add(4 * (size_t)n1), obin = ar.add(4 * (size_t)n1), onm = ar.add(4);
  size_t odec[2], oslot[3], ocnt[3];
  for (int k = 0; k < 2; k++) odec[k] = ar.add(4 * (size_t)n1);
  for (int k = 0; k < 3; k++) oslot[k] = ar.add(8 * INIT_SLOTS * n2s);
  for (int k = 0; k < 3; k++) ocnt[k] = ar.add(4 * n2s);
  const size_t ostate = ar.add(4 * INIT_STATE_INTS);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  uint8_t* A = m->arena;
  orbfe_frame_view d2, d1;
  if ((st = sbp_stage(m, p, f2, f1->descriptors, nullptr, &d2))) return st;  // queries = F1's descriptors
  if ((st = upload_frame(m, o1, f1, &d1))) return st;
  stage_h2d(m, A + oprev, prev_matched, 8 * (size_t)n1);
  if ((st = flush_h2d(m))) return st;
  if (!p.cache) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_for_initialization: F2 too large");
  int32_t* dec[2] = {(int32_t*)(A + odec[0]), (int32_t*)(A + odec[1])};
  int2* slots[3];
  int32_t* cnt[3];
  for (int k = 0; k < 3; k++) {
    slots[k] = (int2*)(A + oslot[k]);
    cnt[k] = (int32_t*)(A + ocnt[k]);
  }
  int32_t* state = (int32_t*)(A + ostate);
  InitQueryArgs qa{n1, n2, d1.keys_un, (const float*)(A + oprev), (float)window_size, (SbpQuery*)(A + p.oq),
                   dec[1], cnt[0], cnt[2], state};
  const int qn = std::max(std::max(n1, n2), INIT_STATE_INTS);
  ORBFE_LAUNCH("k_init_queries", k_init_queries, dim3((qn + 255) / 256), dim3(256), 0, m->stream, qa);
  sbp_launch_round0(m, p, f2, d2, SbpMode{1, TH_LOW, SBP_BLOCK_NONE, 0, 0});
  // the claim order: fixpoint rounds (each exits at once after convergence), then the finish
  InitFixArgs fa;
  std::memset(&fa, 0, sizeof(fa));
  fa.n1 = n1;
  fa.n2 = n2;
  fa.cand_cap = cap;
  fa.nnratio = m->nnratio;
  fa.cand = (const uint32_t*)(A + p.ocand);
  fa.cand_n = (const int32_t*)(A + p.ocand_n);
  fa.state = state;
  const int gx = std::max((n1 + 15) / 16, (n2 + 255) / 256);
  for (int r = 0; r < INIT_MAX_ROUNDS; r++) {
    fa.round = r;
    fa.dec_prev = dec[(r + 1) & 1];
    fa.dec_cur = dec[r & 1];
    fa.slots_prev = slots[(r + 2) % 3];
    fa.cnt_prev = cnt[(r + 2) % 3];
    fa.slots_cur = slots[r % 3];
    fa.cnt_cur = cnt[r % 3];
    fa.cnt_next = cnt[(r + 1) % 3];
    ORBFE_LAUNCH("k_init_round", k_init_round, dim3(gx), dim3(256), 0, m->stream, fa);
  }
  InitSeqArgs sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.n1 = n1;
  sa.n2 = n2;
  sa.cand_cap = cap;
  sa.check_ori = m->check_ori;
  sa.nnratio = m->nnratio;
  sa.cand = fa.cand;
  sa.cand_n = fa.cand_n;
  sa.keys1 = d1.keys_un;
  sa.keys2 = d2.keys_un;
  sa.match12 = (int32_t*)(A + om);
  sa.bin_of = (int32_t*)(A + obin);
  sa.prev = (float*)(A + oprev);
  sa.nmatches = (int32_t*)(A + onm);
  sa.state = state;
  sa.dec[0] = dec[0];
  sa.dec[1] = dec[1];
  for (int k = 0; k < 3; k++) {
    sa.slots[k] = slots[k];
    sa.cnt[k] = cnt[k];
  }
  const size_t lds = sizeof(int) * (2 * n2s + HISTO_LENGTH + 4);
  if (lds > 160 * 1024) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_for_initialization: F2 too large");
  ORBFE_LAUNCH("k_init_seq", k_init_seq, dim3(1), dim3(64), lds, m->stream, sa);
  ORBFE_HIP_CHECK(hipGetLastError());
  int32_t nm = 0;
  orbfe_mi::stage_d2h(m, match12, A + om, 4 * (size_t)n1);
  orbfe_mi::stage_d2h(m, prev_matched, A + oprev, 8 * (size_t)n1);
  orbfe_mi::stage_d2h(m, &nm, A + onm, 4);
  if ((st = orbfe_mi::fetch_d2h(m))) return st;
  *nmatches = nm;
  return ORBFE_OK;
}

extern "C" int orbfe_compute_distinctive_descriptors_device(orbfe_matcher* m, int n_points, const int32_t* d_offsets,
                                                            const uint8_t* d_descriptors, int32_t* d_best_index,
                                                            void* stream) {
  if (!m || n_points < 0 || (n_points > 0 && (!d_offsets || !d_descriptors || !d_best_index)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_distinctive_descriptors_device: bad argument");
  if (n_points == 0) return ORBFE_OK;
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  ORBFE_LAUNCH("k_distinctive", k_distinctive, dim3((n_points + 3) / 4), dim3(256), 0, s, n_points, d_offsets, d_descriptors,
                     d_best_index);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

extern "C" int orbfe_compute_distinctive_descriptors(orbfe_matcher* m, int n_points, const int32_t* offsets,
                                                     const uint8_t* descriptors, int32_t* best_index) {
  if (!m || n_points < 0 || (n_points > 0 && (!offsets || !best_index)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_distinctive_descriptors: bad argument");
  if (n_points == 0) return ORBFE_OK;
  if (offsets[0] != 0) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_distinctive_descriptors: offsets[0] != 0");
  for (int i = 0; i < n_points; i++) {
    const int n = offsets[i + 1] - offsets[i];
    if (n < 0 || n > DD_MAX_OBS)
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_compute_distinctive_descriptors: bad observation count");
  }
  const int total = offsets[n_points];
  if (total > 0 && !descriptors) return orbfe_set_error(ORBFE_ERR_ARG, "descriptors is NULL");
  hipSetDevice(m->device);
  Arena ar;
  const size_t oo = ar.add(4 * (size_t)(n_points + 1)), od = ar.add(32 * (size_t)std::max(total, 1)),
               ob = ar.add(4 * (size_t)n_points);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  uint8_t* A = m->arena;
  stage_h2d(m, A + oo, offsets, 4 * (size_t)(n_points + 1));
  if (total > 0) stage_h2d(m, A + od, descriptors, 32 * (size_t)total);
  if ((st = flush_h2d(m))) return st;
  if ((st = orbfe_compute_distinctive_descriptors_device(m, n_points, (const int32_t*)(A + oo), A + od,
                                                         (int32_t*)(A + ob), m->stream)))
    return st;
  orbfe_mi::stage_d2h(m, best_index, A + ob, 4 * (size_t)n_points);
  return orbfe_mi::fetch_d2h(m);
}
