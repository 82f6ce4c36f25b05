// orbfe_vocab.hip -- the DBoW2 ORB vocabulary on gfx950: loaders, and transform of descriptor
// sets into BowVector + FeatureVector.
//
// Reference (Thirdparty/DBoW2/DBoW2/):
//   TemplatedVocabulary.h:1140-1207  transform(features, BowVector, FeatureVector, levelsup)
//   TemplatedVocabulary.h:1231-1272  descent of one descriptor: at every level the child with the
//                                    smallest FORB::distance, strict '<' (the first best child
//                                    wins); the node reached at level m_L - levelsup is the
//                                    FeatureVector node; word id + weight of the final node
//   BowVector.cpp:35-85              addWeight (TF, TF_IDF) / addIfNotExist (IDF, BINARY),
//                                    normalize (L1: sum of |w|, L2: sqrt of the sum of squares,
//                                    both in word order; divide when > 0)
//   TemplatedVocabulary.h:1351-1440  loadFromTextFile
//   TemplatedVocabulary.h:1467-1511  loadFromBinaryFile
// Callers: KeyFrame::ComputeBoW (KeyFrame.cc:59-68) and Frame::ComputeBoW (Frame.cc:447-454),
// levelsup = 4; SearchByBoW / SearchForTriangulation consume the FeatureVector.
//
// Device layout: every node except the root is a 48-byte child record {descriptor, node id,
// its own children's slot range, weight>0 flag, word id}, stored grouped by parent (siblings
// contiguous, in the reference's push_back order). One dependent load per level: the 16 lanes
// of a descriptor's group each read one sibling record (a group reads 10 x 48 B contiguous at
// k=10), popcount the xor, and a 16-lane min of (distance << 23 | sibling) picks the first best
// child together with everything the next level needs.
//
// k_vocab (two workgroups per image, VOCAB_THREADS each) sorts, in one, the (node, feature) keys into the
// FeatureVector CSR (std::map<NodeId, vector<unsigned>> iteration order) and, in the other, the
// (word, feature) keys into the BowVector: per word the weights are added in feature order
// (addWeight) or the first kept (addIfNotExist); wave 0 sums the norm in word order, the
// workgroup divides. The sorts are bitonic in registers (bitonic_reg).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_vocab.h"
#include "orbfe_device.h"
#include "orbfe_ktimer.h"

#define VOCAB_MAX_FEATURES 8192
#define VOCAB_MAX_CHILDREN (1 << 23)  // sibling index field of the min key
// k_vocab workgroup size. 512: beside the extraction kernels smaller workgroups find room sooner
// (bench 81.4k at 512 or 256 vs 78.7k at 1024); alone 66 / 81 / 61 us
#define VOCAB_THREADS 512

struct __attribute__((aligned(16))) VocRec {
  uint4 d0, d1;       // the node's descriptor (32 B)
  int32_t node;       // node id
  int32_t beg;        // first child slot of this node
  uint32_t cnt;       // number of children | (weight > 0) << 31
  uint32_t word;      // Node::word_id (0 for nodes that are not words)
};
static_assert(sizeof(VocRec) == 48, "child record is 48 bytes");

// normalisation applied after the weights are accumulated (transform :1176-1206)
enum { NORM_L1 = 0, NORM_L2 = 1, NORM_DIV_SIZE = 2, NORM_NONE = 3 };

struct orbfe_vocabulary {
  int device = 0;
  int n_nodes = 0, n_words = 0, k = 0, levels = 0, scoring = 0, weighting = 0;
  int root_beg = 0, root_cnt = 0;
  // host copy of the node table (orbfe_vocab_export)
  std::vector<int32_t> parent;
  std::vector<uint8_t> is_leaf;
  std::vector<uint8_t> desc;
  std::vector<double> weight;
  std::vector<uint32_t> word_id;
  VocRec* d_rec = nullptr;
  double* d_weight = nullptr;
  hipStream_t stream = nullptr;
  // scratch
  uint8_t* d_scratch = nullptr;  // host-call staging
  size_t scratch_bytes = 0;
  // FeatureVector keys, BowVector keys, leaf node per feature: one buffer per launch stream, so
  // that transforms enqueued on different streams may run concurrently
  struct KeyScratch {
    hipStream_t stream;
    unsigned long long* d_keys;
    size_t bytes;
  };
  std::vector<KeyScratch> keys;
};

struct VocabArgs {
  const VocRec* rec;
  const double* weight;
  int root_beg, root_cnt;
  int nid_level;
  int empty;                 // the vocabulary has no words: transform returns empty vectors
  const uint8_t* desc;
  long long desc_stride;     // bytes between images
  const int32_t* counts;     // per image feature count (device)
  int fixed_count;           // used when counts == NULL
  uint32_t* node_ids;
  int32_t* offsets;
  int32_t* indices;
  int32_t* n_nodes;
  uint32_t* bow_words;       // NULL: FeatureVector only
  double* bow_weights;
  int32_t* bow_n;
  int additive;              // TF / TF_IDF: addWeight; IDF / BINARY: addIfNotExist
  int norm_kind;
  int cap;
};

__device__ __forceinline__ uint32_t min16(uint32_t v) {
  v = min(v, (uint32_t)__shfl_xor((int)v, 8, 16));
  v = min(v, (uint32_t)__shfl_xor((int)v, 4, 16));
  v = min(v, (uint32_t)__shfl_xor((int)v, 2, 16));
  v = min(v, (uint32_t)__shfl_xor((int)v, 1, 16));
  return v;
}

// k_vocab_descend: 16 lanes per descriptor, 16 descriptors per workgroup
// (TemplatedVocabulary.h:1231-1272). Writes the (node, feature) and (word, feature) keys, ~0 for
// a stopped word (weight 0, :1171) or an empty slot, and the final node (for its weight).
__global__ __launch_bounds__(256) void k_vocab_descend(VocabArgs a, unsigned long long* fvkeys,
                                                       unsigned long long* bowkeys, int32_t* leaves) {
  const int img = blockIdx.y;
  const int g = threadIdx.x >> 4, sub = threadIdx.x & 15;
  const int i = blockIdx.x * 16 + g;
  if (i >= a.cap) return;  // uniform per 16-lane group
  const int n = min(a.counts ? a.counts[img] : a.fixed_count, a.cap);
  unsigned long long fk = ~0ull, bk = ~0ull;
  int leaf = -1;
  if (i < n && !a.empty) {
    const uint8_t* dp = a.desc + (long long)img * a.desc_stride + (size_t)i * 32;
    uint4 d0, d1;
    load_desc(dp, d0, d1);
    int beg = a.root_beg, node = 0, level = 0, nid = 0;
    uint32_t cntf = (uint32_t)a.root_cnt, word = 0;
    while ((cntf & 0x7fffffffu) != 0) {
      ++level;
      const int nc = (int)(cntf & 0x7fffffffu);
      uint32_t best = 0xffffffffu;
      int bnode = 0, bbeg = 0;
      uint32_t bcnt = 0, bword = 0;
      for (int c0 = 0; c0 < nc; c0 += 16) {
        const int c = c0 + sub;
        if (c < nc) {
          const VocRec* r = a.rec + beg + c;
          const uint4 r0 = r->d0, r1 = r->d1;
          const int4 meta = *reinterpret_cast<const int4*>(&r->node);
          const uint32_t key = ((uint32_t)hamming256(d0, d1, r0, r1) << 23) | (uint32_t)c;
          if (key < best) {  // this lane's siblings ascend: strict keeps the first best
            best = key;
            bnode = meta.x;
            bbeg = meta.y;
            bcnt = (uint32_t)meta.z;
            bword = (uint32_t)meta.w;
          }
        }
      }
      const uint32_t m = min16(best);  // smallest distance, then the smallest sibling index
      const int src = (int)(threadIdx.x & 48u) + (int)((m & 0x7fffffu) & 15u);
      node = __shfl(bnode, src, 64);
      beg = __shfl(bbeg, src, 64);
      cntf = (uint32_t)__shfl((int)bcnt, src, 64);
      word = (uint32_t)__shfl((int)bword, src, 64);
      if (level == a.nid_level) nid = node;
    }
    // the reference leaves nid unset when the descent ends above nid_level:
    // the final node stands in
    if (level < a.nid_level) nid = node;
    if (cntf >> 31) {  // weight > 0: not stopped
      fk = ((unsigned long long)(uint32_t)nid << 32) | (uint32_t)i;
      bk = ((unsigned long long)word << 32) | (uint32_t)i;
    }
    leaf = node;
  }
  if (sub == 0) {
    const long long o = (long long)img * a.cap + i;
    fvkeys[o] = fk;
    bowkeys[o] = bk;
    leaves[o] = leaf;
  }
}

// Ascending bitonic sort of P2 = VOCAB_THREADS E keys held in registers: element
// e = (wave * E + r) * 64 + lane is register r of that lane, so a wave owns 64 E consecutive keys.
// Stages with j < 64 swap across lanes (ds_bpermute), 64 <= j < 64 E across a lane's registers,
// and only j >= 64 E go through LDS with barriers. The keys come from and return to ka (the LDS
// array the rest of k_vocab reads).
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ unsigned long long cx_keep(unsigned long long me, unsigned long long other, int e, int j,
                                                      int k) {
  const bool lower = (e & j) == 0, asc = (e & k) == 0;
  return (lower == asc) ? (other < me ? other : me) : (other > me ? other : me);
}
__device__ __forceinline__ void cx_pair(unsigned long long& lo, unsigned long long& hi, bool asc) {
  const unsigned long long a = lo, b = hi;
  const bool sw = asc ? (a > b) : (a < b);
  lo = sw ? b : a;
  hi = sw ? a : b;
}

template <int E>
__device__ __forceinline__ void bitonic_reg(unsigned long long* ka) {
  constexpr int P2 = VOCAB_THREADS * E;
  const int l = lane_id(), w = wave_id();
  unsigned long long va[E];
#pragma unroll
  for (int r = 0; r < E; r++) va[r] = ka[(w * E + r) * 64 + l];
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64 * E) {  // across waves
        __syncthreads();  // the previous such stage's partner reads are done
#pragma unroll
        for (int r = 0; r < E; r++) ka[(w * E + r) * 64 + l] = va[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; r++) {
          const int e = (w * E + r) * 64 + l;
          va[r] = cx_keep(va[r], ka[e ^ j], e, j, k);
        }
      } else if (j >= 64) {  // across this lane's registers (static indices per q)
        const int jr = j >> 6;
#pragma unroll
        for (int q = 1; q < E; q <<= 1) {
          if (jr == q) {
#pragma unroll
            for (int r = 0; r < E; r++)
              if ((r & q) == 0) cx_pair(va[r], va[r | q], ((((w * E + r) * 64 + l) & k) == 0));
          }
        }
      } else {  // across lanes
#pragma unroll
        for (int r = 0; r < E; r++) {
          const int e = (w * E + r) * 64 + l;
          va[r] = cx_keep(va[r], shfl_xor_u64(va[r], j), e, j, k);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < E; r++) ka[(w * E + r) * 64 + l] = va[r];
  __syncthreads();
}

// ascending bitonic sort of P2 keys through LDS, one compare-exchange per thread per stage
// (rounds 1-3's sort; ORBFE_VOCAB_LDS_SORT selects it)
__device__ __forceinline__ void bitonic_lds(unsigned long long* skeys, int P2) {
  const int t = threadIdx.x;
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int pidx = t; pidx < (P2 >> 1); pidx += VOCAB_THREADS) {
        const int i = ((pidx & ~(j - 1)) << 1) | (pidx & (j - 1)), ixj = i + j;  // j is a power of 2
        const unsigned long long x = skeys[i], y = skeys[ixj];
        if ((i & k) == 0 ? (x > y) : (x < y)) {
          skeys[i] = y;
          skeys[ixj] = x;
        }
      }
      __syncthreads();
    }
  }
}

// P2 a power of two from VOCAB_THREADS to VOCAB_MAX_FEATURES (k_vocab pads to at least one key
// per thread)
__device__ __forceinline__ void sort_keys(unsigned long long* ka, int P2) {
  const int E = P2 / VOCAB_THREADS;
  if (E <= 1)
    bitonic_reg<1>(ka);
  else if (E == 2)
    bitonic_reg<2>(ka);
  else if (E == 4)
    bitonic_reg<4>(ka);
  else if (E == 8)
    bitonic_reg<8>(ka);
  else  // more than 8 keys per thread (large nfeatures at small workgroups): through LDS
    bitonic_lds(ka, P2);
}

// Starts of the runs of equal key>>32 among the nv sorted valid keys: every thread owns a
// contiguous chunk; returns this thread's first output position and the total run count.
__device__ __forceinline__ int2 run_starts(const unsigned long long* skeys, int nv, int beg, int end,
                                          int* s_wsum) {
  int cnt = 0;
  for (int i = beg; i < end; i++)
    cnt += i == 0 || (uint32_t)(skeys[i] >> 32) != (uint32_t)(skeys[i - 1] >> 32);
  const int lane = lane_id(), w = wave_id();
  int inc = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_wsum[w] = inc;
  __syncthreads();
  int pos = inc - cnt;
  for (int k = 0; k < w; k++) pos += s_wsum[k];
  int runs = 0;
  for (int k = 0; k < VOCAB_THREADS / 64; k++) runs += s_wsum[k];
  __syncthreads();  // s_wsum is reused by the next call
  return make_int2(pos, runs);
}

// ((0 + f(v[0])) + f(v[1])) + ... over v[0..nw), f = |x| or x*x, one thread; v is readable and
// zero from nw to nw + 3H (k_vocab zeroes 128 slots)
template <bool L2>
__device__ __forceinline__ double ordered_sum(const double* v, int nw) {
  constexpr int H = 16;  // words per register set (2 H doubles)
  double A[H], B[H], s = 0.0;
#pragma unroll
  for (int i = 0; i < H; i++) A[i] = v[i];
  for (int j0 = 0; j0 < nw; j0 += 2 * H) {
#pragma unroll
    for (int i = 0; i < H; i++) B[i] = v[j0 + H + i];
#pragma unroll
    for (int i = 0; i < H; i++) s += L2 ? A[i] * A[i] : fabs(A[i]);
#pragma unroll
    for (int i = 0; i < H; i++) A[i] = v[j0 + 2 * H + i];
#pragma unroll
    for (int i = 0; i < H; i++) s += L2 ? B[i] * B[i] : fabs(B[i]);
  }
  return s;
}

// One vector of one image: fv -- the FeatureVector from the (node, feature) keys; else the
// BowVector from the (word, feature) keys. skeys: P2 keys, then P2 + 128 doubles.
__device__ __forceinline__ void vocab_part(const VocabArgs& a, bool fv, int img, int n, int P2,
                                           const unsigned long long* fvkeys,
                                           const unsigned long long* bowkeys, const int32_t* leaves,
                                           unsigned long long* skeys, int* s_n, int* s_wsum, double* s_norm) {
  const int t = threadIdx.x;
  const long long kbase = (long long)img * a.cap;
  const unsigned long long* src = fv ? fvkeys : bowkeys;
  for (int i = t; i < P2; i += VOCAB_THREADS) skeys[i] = i < n ? src[kbase + i] : ~0ull;
  if (t == 0) *s_n = 0;
  __syncthreads();
  sort_keys(skeys, P2);  // stable: the feature index is the low half of every key
  int nvalid = 0;
  for (int i = t; i < n; i += VOCAB_THREADS) nvalid += skeys[i] != ~0ull;
  nvalid = wave_sum(nvalid);
  if (lane_id() == 0) atomicAdd(s_n, nvalid);
  __syncthreads();
  const int nv = *s_n;  // valid keys sort first; the stopped set is the same for both vectors
  const int per = (nv + VOCAB_THREADS - 1) / VOCAB_THREADS;
  const int beg = min(t * per, nv), end = min(beg + per, nv);
  if (fv) {
    uint32_t* ids = a.node_ids + kbase;
    int32_t* offs = a.offsets + (long long)img * (a.cap + 1);
    int32_t* idx = a.indices + kbase;
    for (int i = t; i < nv; i += VOCAB_THREADS) idx[i] = (int32_t)(skeys[i] & 0xffffffffull);
    const int2 pr = run_starts(skeys, nv, beg, end, s_wsum);
    int pos = pr.x;
    for (int i = beg; i < end; i++) {
      if (i == 0 || (uint32_t)(skeys[i] >> 32) != (uint32_t)(skeys[i - 1] >> 32)) {
        ids[pos] = (uint32_t)(skeys[i] >> 32);
        offs[pos] = i;
        pos++;
      }
    }
    if (t == 0) {
      offs[pr.y] = nv;
      a.n_nodes[img] = pr.y;
    }
    return;
  }
  double* sval = reinterpret_cast<double*>(skeys + P2);
  uint32_t* words = a.bow_words + kbase;
  double* wout = a.bow_weights + kbase;
  const int2 pr = run_starts(skeys, nv, beg, end, s_wsum);
  const int nw = pr.y;
  int pos = pr.x;
  for (int i = beg; i < end; i++) {
    const uint32_t word = (uint32_t)(skeys[i] >> 32);
    if (i != 0 && word == (uint32_t)(skeys[i - 1] >> 32)) continue;
    // BowVector::addWeight (BowVector.cpp:35-47): insert w, then += w per later feature in
    // feature order; addIfNotExist (:51-59): the first feature's weight only
    double s = a.weight[leaves[kbase + (int)(skeys[i] & 0xffffffffull)]];
    if (a.additive)
      for (int j = i + 1; j < nv && (uint32_t)(skeys[j] >> 32) == word; j++)
        s += a.weight[leaves[kbase + (int)(skeys[j] & 0xffffffffull)]];
    words[pos] = word;
    sval[pos] = s;
    pos++;
  }
  __syncthreads();
  // zero the slots the norm loop reads past nw (up to 128 beyond; the LDS holds P2 + 128 doubles)
  for (int j = nw + t; j < nw + 128; j += VOCAB_THREADS) sval[j] = 0.0;
  __syncthreads();
  if (t == 0) {
    // BowVector::normalize (BowVector.cpp:63-85): the norm accumulates in word order -- one
    // dependent add per word. Thread 0 reads the words ahead from LDS into registers (two
    // alternating sets), so the chain is one v_add_f64 per word (|w| as a source modifier); the
    // zero slots past nw add nothing (norm + 0 == norm, norm >= 0).
    double norm = 0.0;
    const bool sum = a.norm_kind == NORM_L1 || a.norm_kind == NORM_L2;
    if (sum) {
      if (a.norm_kind == NORM_L2)
        norm = sqrt(ordered_sum<true>(sval, nw));
      else
        norm = ordered_sum<false>(sval, nw);
    } else if (a.norm_kind == NORM_DIV_SIZE) {
      norm = (double)nw;  // transform :1176-1182, "unnecessary when normalizing"
    }
    *s_norm = norm;
    a.bow_n[img] = nw;
  }
  __syncthreads();
  const double norm = *s_norm;
  const bool divide = a.norm_kind != NORM_NONE && norm > 0.0;
  for (int j = t; j < nw; j += VOCAB_THREADS) wout[j] = divide ? sval[j] / norm : sval[j];
}

// Two workgroups per image (blockIdx.y 0: FeatureVector, 1: BowVector; one workgroup doing both
// in turn measured slower)
__global__ __launch_bounds__(VOCAB_THREADS) void k_vocab(VocabArgs a, const unsigned long long* fvkeys,
                                                         const unsigned long long* bowkeys,
                                                         const int32_t* leaves) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];  // P2 keys, then P2 + 128 doubles
  __shared__ int s_n;
  __shared__ int s_wsum[VOCAB_THREADS / 64];
  __shared__ double s_norm;
  const int img = blockIdx.x;
  const int n = a.empty ? 0 : min(a.counts ? a.counts[img] : a.fixed_count, a.cap);
  int P2 = VOCAB_THREADS;  // sort_keys' smallest size: one key per thread
  while (P2 < n) P2 <<= 1;
  vocab_part(a, blockIdx.y == 0, img, n, P2, fvkeys, bowkeys, leaves, skeys, &s_n, s_wsum, &s_norm);
}

// ------------------------------------------------------------------------------------------
// host: the node table -> device records

static int vocab_build(orbfe_vocabulary* v, int device) {
  const int N = v->n_nodes;
  // word ids in node order, as both loaders assign them (m_words.size() at the leaf's line)
  v->word_id.assign(N, 0u);
  int nw = 0;
  for (int i = 1; i < N; i++)
    if (v->is_leaf[i]) v->word_id[i] = (uint32_t)nw++;
  v->n_words = nw;
  // children grouped by parent, ascending id (push_back order)
  std::vector<int32_t> cnt(N + 1, 0), off(N + 1, 0);
  for (int i = 1; i < N; i++) cnt[v->parent[i]]++;
  for (int p = 0; p < N; p++) {
    if (cnt[p] >= VOCAB_MAX_CHILDREN)
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab: a node has >= 2^23 children");
    off[p + 1] = off[p] + cnt[p];
  }
  std::vector<int32_t> fill(off.begin(), off.end() - 1);
  std::vector<VocRec> rec(N > 1 ? N - 1 : 1);
  for (int i = 1; i < N; i++) {
    VocRec& r = rec[fill[v->parent[i]]++];
    memcpy(&r.d0, &v->desc[(size_t)i * 32], 16);
    memcpy(&r.d1, &v->desc[(size_t)i * 32 + 16], 16);
    r.node = i;
    r.beg = off[i];
    r.cnt = (uint32_t)cnt[i] | (v->weight[i] > 0 ? 0x80000000u : 0u);
    r.word = v->word_id[i];
  }
  v->root_beg = off[0];
  v->root_cnt = cnt[0];
  v->device = device;
  if (device < 0) return ORBFE_OK;  // host-only table (loaders / export; no transform)
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_vocab: no such HIP device");
  v->device = device;
  ORBFE_HIP_CHECK(hipSetDevice(device));
  ORBFE_HIP_CHECK(hipMalloc(&v->d_rec, sizeof(VocRec) * rec.size()));
  ORBFE_HIP_CHECK(hipMalloc(&v->d_weight, sizeof(double) * (size_t)N));
  ORBFE_HIP_CHECK(hipMemcpy(v->d_rec, rec.data(), sizeof(VocRec) * rec.size(), hipMemcpyHostToDevice));
  ORBFE_HIP_CHECK(hipMemcpy(v->d_weight, v->weight.data(), sizeof(double) * (size_t)N, hipMemcpyHostToDevice));
  ORBFE_HIP_CHECK(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
  // k_vocab holds up to 8192 keys + 8192 + 128 weights in LDS (129 KiB of the CU's 160 KiB)
  ORBFE_HIP_CHECK(hipFuncSetAttribute((const void*)k_vocab, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      2 * sizeof(unsigned long long) * VOCAB_MAX_FEATURES + 128 * sizeof(double)));
  return ORBFE_OK;
}

// The parent table must describe a tree rooted at node 0 (the reference indexes m_nodes[pid]
// unchecked; a cycle would make its descent loop forever).
static bool vocab_acyclic(const std::vector<int32_t>& parent) {
  const int N = (int)parent.size();
  std::vector<uint8_t> state(N, 0);  // 0 unknown, 1 on the current path, 2 reaches the root
  state[0] = 2;
  std::vector<int> path;
  for (int i = 1; i < N; i++) {
    int u = i;
    path.clear();
    while (state[u] == 0) {
      state[u] = 1;
      path.push_back(u);
      u = parent[u];
    }
    if (state[u] == 1) return false;
    for (int x : path) state[x] = 2;
  }
  return true;
}

static int vocab_finish(orbfe_vocabulary* v, int device, orbfe_vocabulary** out) {
  if (!vocab_acyclic(v->parent)) {
    delete v;
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab: the parent table is not a tree");
  }
  const int st = vocab_build(v, device);
  if (st != ORBFE_OK) {
    orbfe_vocab_destroy(v);
    return st;
  }
  *out = v;
  return ORBFE_OK;
}

static bool vocab_header_ok(int k, int L, int scoring, int weighting) {
  // loadFromTextFile :1374 accepts these ranges
  return !(k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
           weighting > 3);
}

extern "C" int orbfe_vocab_create(int n_nodes, int k, int levels, int scoring, int weighting,
                                  const int32_t* parent, const uint8_t* is_leaf,
                                  const uint8_t* node_desc, const double* weights, int device,
                                  orbfe_vocabulary** out) {
  if (!out || n_nodes <= 0 || !parent || !is_leaf || !node_desc || !weights ||
      !vocab_header_ok(k, levels, scoring, weighting))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_create: bad argument");
  *out = nullptr;
  for (int i = 1; i < n_nodes; i++)
    if (parent[i] < 0 || parent[i] >= n_nodes || parent[i] == i)
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_create: parent out of range");
  orbfe_vocabulary* v = new orbfe_vocabulary();
  v->n_nodes = n_nodes;
  v->k = k;
  v->levels = levels;
  v->scoring = scoring;
  v->weighting = weighting;
  v->parent.assign(parent, parent + n_nodes);
  v->parent[0] = -1;
  v->is_leaf.resize(n_nodes);
  for (int i = 0; i < n_nodes; i++) v->is_leaf[i] = i > 0 && is_leaf[i] ? 1 : 0;
  v->desc.assign(node_desc, node_desc + (size_t)n_nodes * 32);
  v->weight.assign(weights, weights + n_nodes);
  return vocab_finish(v, device, out);
}

// loadFromTextFile (TemplatedVocabulary.h:1351-1440). Line parsing follows the stream
// extractions: parent, is-leaf flag, FORB::L = 32 byte values (FORB::fromString, FORB.cpp:120-135:
// int, stored as unsigned char), the weight (double).
extern "C" int orbfe_vocab_load_text(const char* path, int device, orbfe_vocabulary** out) {
  if (!path || !out) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_text: bad argument");
  *out = nullptr;
  std::ifstream f(path);
  if (!f.is_open()) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_text: cannot open file");
  std::string line;
  if (!std::getline(f, line)) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_text: empty file");
  int k = -1, L = -1, sc = -1, wt = -1;
  if (sscanf(line.c_str(), "%d %d %d %d", &k, &L, &sc, &wt) != 4 || !vocab_header_ok(k, L, sc, wt))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_text: not a vocabulary text file");
  orbfe_vocabulary* v = new orbfe_vocabulary();
  v->k = k;
  v->levels = L;
  v->scoring = sc;
  v->weighting = wt;
  v->parent.push_back(-1);
  v->is_leaf.push_back(0);
  v->desc.resize(32, 0);
  v->weight.push_back(0.0);
  auto bad = [&](const char* why) {
    delete v;
    return orbfe_set_error(ORBFE_ERR_ARG, why);
  };
  while (std::getline(f, line)) {
    const char* p = line.c_str();
    char* e = nullptr;
    while (*p == ' ' || *p == '\t' || *p == '\r') p++;
    if (!*p) continue;  // no token on the line: skipped (the reference reads an unset parent)
    const int nid = (int)v->parent.size();
    const long pid = strtol(p, &e, 10);
    if (e == p || pid < 0 || pid >= nid) return bad("orbfe_vocab_load_text: bad parent id");
    p = e;
    const long leaf = strtol(p, &e, 10);
    if (e == p) return bad("orbfe_vocab_load_text: bad leaf flag");
    p = e;
    uint8_t d[32];
    for (int b = 0; b < 32; b++) {
      const long x = strtol(p, &e, 10);
      if (e == p) return bad("orbfe_vocab_load_text: short descriptor");
      d[b] = (uint8_t)x;  // (unsigned char)n
      p = e;
    }
    const double w = strtod(p, &e);
    if (e == p) return bad("orbfe_vocab_load_text: missing weight");
    v->parent.push_back((int32_t)pid);
    v->is_leaf.push_back(leaf > 0 ? 1 : 0);
    v->desc.insert(v->desc.end(), d, d + 32);
    v->weight.push_back(w);
  }
  v->n_nodes = (int)v->parent.size();
  return vocab_finish(v, device, out);
}

// loadFromBinaryFile (TemplatedVocabulary.h:1467-1511): header nb_nodes, size_node, k, L, scoring,
// weighting (4 bytes each); per node int parent, 32 descriptor bytes, float weight, bool leaf at
// byte 40. The loop tests eof before the read that hits it, so after the last record it runs once
// more on the unchanged buffer: node nb_nodes is a copy of node nb_nodes - 1.
extern "C" int orbfe_vocab_load_binary(const char* path, int device, orbfe_vocabulary** out) {
  if (!path || !out) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_binary: bad argument");
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_binary: cannot open file");
  uint32_t hdr[6];
  std::vector<uint8_t> body;
  const bool hdr_ok = fread(hdr, 4, 6, f) == 6;
  if (hdr_ok) {
    uint8_t buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) body.insert(body.end(), buf, buf + got);
  }
  fclose(f);
  if (!hdr_ok) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_binary: short header");
  const uint32_t nb_nodes = hdr[0], size_node = hdr[1];
  const int k = (int)hdr[2], L = (int)hdr[3], sc = (int)hdr[4], wt = (int)hdr[5];
  if (size_node < 41 || nb_nodes < 2 || !vocab_header_ok(k, L, sc, wt) ||
      body.size() != (size_t)(nb_nodes - 1) * size_node)
    return orbfe_set_error(ORBFE_ERR_ARG,
                           "orbfe_vocab_load_binary: not a vocabulary binary file (record count or size)");
  orbfe_vocabulary* v = new orbfe_vocabulary();
  v->k = k;
  v->levels = L;
  v->scoring = sc;
  v->weighting = wt;
  const int N = (int)nb_nodes + 1;
  v->n_nodes = N;
  v->parent.assign(N, -1);
  v->is_leaf.assign(N, 0);
  v->desc.assign((size_t)N * 32, 0);
  v->weight.assign(N, 0.0);
  for (int nid = 1; nid < N; nid++) {
    const uint8_t* r = body.data() + (size_t)(nid < (int)nb_nodes ? nid - 1 : nb_nodes - 2) * size_node;
    int32_t pid;
    float w;
    memcpy(&pid, r, 4);
    memcpy(&w, r + 36, 4);
    if (pid < 0 || pid >= N || pid == nid) {
      delete v;
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_load_binary: bad parent id");
    }
    v->parent[nid] = pid;
    memcpy(&v->desc[(size_t)nid * 32], r + 4, 32);
    v->weight[nid] = (double)w;
    v->is_leaf[nid] = r[40] ? 1 : 0;
  }
  return vocab_finish(v, device, out);
}

extern "C" int orbfe_vocab_get_info(const orbfe_vocabulary* v, orbfe_vocab_info* info) {
  if (!v || !info) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_get_info: bad argument");
  info->n_nodes = v->n_nodes;
  info->n_words = v->n_words;
  info->k = v->k;
  info->levels = v->levels;
  info->scoring = v->scoring;
  info->weighting = v->weighting;
  return ORBFE_OK;
}

extern "C" int orbfe_vocab_export(const orbfe_vocabulary* v, int32_t* parent, uint8_t* is_leaf,
                                  uint8_t* node_desc, double* weights, uint32_t* word_id) {
  if (!v) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_export: bad argument");
  const size_t N = (size_t)v->n_nodes;
  if (parent) memcpy(parent, v->parent.data(), 4 * N);
  if (is_leaf) memcpy(is_leaf, v->is_leaf.data(), N);
  if (node_desc) memcpy(node_desc, v->desc.data(), 32 * N);
  if (weights) memcpy(weights, v->weight.data(), 8 * N);
  if (word_id) memcpy(word_id, v->word_id.data(), 4 * N);
  return ORBFE_OK;
}

extern "C" int orbfe_vocab_destroy(orbfe_vocabulary* v) {
  if (!v) return ORBFE_OK;
  if (v->device < 0) {
    delete v;
    return ORBFE_OK;
  }
  hipSetDevice(v->device);
  if (v->stream) hipStreamSynchronize(v->stream);
  hipFree(v->d_rec);
  hipFree(v->d_weight);
  hipFree(v->d_scratch);
  for (auto& k : v->keys) hipFree(k.d_keys);
  if (v->stream) hipStreamDestroy(v->stream);
  delete v;
  return ORBFE_OK;
}

static int launch_vocab(orbfe_vocabulary* v, int n_images, const uint8_t* d_desc, size_t desc_stride,
                        const int32_t* d_counts, int fixed_count, int levelsup, uint32_t* d_bow_words,
                        double* d_bow_weights, int32_t* d_bow_n, uint32_t* d_node_ids,
                        int32_t* d_offsets, int32_t* d_indices, int32_t* d_n_nodes, int cap,
                        hipStream_t s) {
  if (cap <= 0 || cap > VOCAB_MAX_FEATURES)
    return orbfe_set_error(ORBFE_ERR_ARG, "vocab transform: cap must be in 1..8192");
  VocabArgs a;
  a.rec = v->d_rec;
  a.weight = v->d_weight;
  a.root_beg = v->root_beg;
  a.root_cnt = v->root_cnt;
  a.nid_level = v->levels - levelsup;
  a.empty = v->n_words == 0;  // TemplatedVocabulary::empty()
  a.desc = d_desc;
  a.desc_stride = (long long)desc_stride;
  a.counts = d_counts;
  a.fixed_count = fixed_count;
  a.node_ids = d_node_ids;
  a.offsets = d_offsets;
  a.indices = d_indices;
  a.n_nodes = d_n_nodes;
  a.bow_words = d_bow_words;
  a.bow_weights = d_bow_weights;
  a.bow_n = d_bow_n;
  a.additive = v->weighting == ORBFE_VOC_TF || v->weighting == ORBFE_VOC_TF_IDF;
  const bool must = v->scoring != ORBFE_VOC_DOT_PRODUCT;  // ScoringObject.h:73-88
  a.norm_kind = must ? (v->scoring == ORBFE_VOC_L2_NORM ? NORM_L2 : NORM_L1)
                     : (a.additive ? NORM_DIV_SIZE : NORM_NONE);
  a.cap = cap;
  int P2 = 1;
  while (P2 < cap) P2 <<= 1;
  const size_t slots = (size_t)cap * n_images;
  const size_t need = slots * (2 * sizeof(unsigned long long) + sizeof(int32_t));
  orbfe_vocabulary::KeyScratch* ks = nullptr;
  for (auto& k : v->keys)
    if (k.stream == s) ks = &k;
  if (!ks) {
    v->keys.push_back({s, nullptr, 0});
    ks = &v->keys.back();
  }
  if (need > ks->bytes) {
    hipFree(ks->d_keys);  // synchronises the device: no launch still reads it
    ks->d_keys = nullptr;
    ks->bytes = 0;
    ORBFE_HIP_CHECK(hipMalloc(&ks->d_keys, need));
    ks->bytes = need;
  }
  unsigned long long* fvk = ks->d_keys;
  unsigned long long* bwk = fvk + slots;
  int32_t* leaves = reinterpret_cast<int32_t*>(bwk + slots);
  // P2 keys, then (BowVector workgroups) P2 doubles
  P2 = P2 < VOCAB_THREADS ? VOCAB_THREADS : P2;  // k_vocab sorts at least one key per thread
  const size_t lds = sizeof(unsigned long long) * P2 + (d_bow_words ? sizeof(double) * (P2 + 128) : 0);
  ORBFE_LAUNCH("k_vocab_descend", k_vocab_descend, dim3((cap + 15) / 16, n_images), dim3(256), 0, s, a, fvk, bwk, leaves);
  ORBFE_LAUNCH("k_vocab", k_vocab, dim3(n_images, d_bow_words ? 2 : 1), dim3(VOCAB_THREADS), lds, s, a,
                     (const unsigned long long*)fvk,
                     (const unsigned long long*)bwk, (const int32_t*)leaves);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

extern "C" int orbfe_vocab_transform_batch_device(orbfe_vocabulary* v, int n_images,
                                                  const uint8_t* d_desc, size_t desc_stride,
                                                  const int32_t* d_counts, int levelsup,
                                                  uint32_t* d_bow_words, double* d_bow_weights,
                                                  int32_t* d_bow_n, uint32_t* d_node_ids,
                                                  int32_t* d_offsets, int32_t* d_indices,
                                                  int32_t* d_n_nodes, int cap, void* stream) {
  const bool bow_any = d_bow_words || d_bow_weights || d_bow_n;
  const bool bow_all = d_bow_words && d_bow_weights && d_bow_n;
  if (v && v->device < 0) return orbfe_set_error(ORBFE_ERR_STATE, "vocabulary loaded host-only (device < 0)");
  if (!v || n_images < 0 || (bow_any && !bow_all) ||
      (n_images > 0 && (!d_desc || !d_counts || !d_node_ids || !d_offsets || !d_indices || !d_n_nodes)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_transform_batch_device: bad argument");
  if (n_images == 0) return ORBFE_OK;
  hipSetDevice(v->device);
  return launch_vocab(v, n_images, d_desc, desc_stride, d_counts, 0, levelsup, d_bow_words,
                      d_bow_weights, d_bow_n, d_node_ids, d_offsets, d_indices, d_n_nodes, cap,
                      stream ? (hipStream_t)stream : v->stream);
}

extern "C" int orbfe_vocab_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                                     uint32_t* bow_words, double* bow_weights, int* n_words,
                                     uint32_t* node_ids, int32_t* offsets, int32_t* indices,
                                     int* n_nodes) {
  const bool bow = bow_words || bow_weights || n_words;
  if (!v || n < 0 || !n_nodes || (bow && !(bow_words && bow_weights && n_words)) ||
      (n > 0 && (!desc || !node_ids || !offsets || !indices)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_transform: bad argument");
  if (n == 0) {
    *n_nodes = 0;
    if (offsets) offsets[0] = 0;
    if (bow) *n_words = 0;
    return ORBFE_OK;
  }
  if (n > VOCAB_MAX_FEATURES) return orbfe_set_error(ORBFE_ERR_ARG, "too many descriptors");
  if (v->device < 0) return orbfe_set_error(ORBFE_ERR_STATE, "vocabulary loaded host-only (device < 0)");
  hipSetDevice(v->device);
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_desc = al((size_t)n * 32), b_i = al((size_t)n * 4 + 4), b_d = al((size_t)n * 8);
  const size_t need = b_desc + 4 * b_i + b_d + 256;
  if (need > v->scratch_bytes) {
    hipFree(v->d_scratch);
    v->d_scratch = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&v->d_scratch, need));
    v->scratch_bytes = need;
  }
  uint8_t* dd = v->d_scratch;
  uint32_t* did = (uint32_t*)(dd + b_desc);
  int32_t* doff = (int32_t*)(dd + b_desc + b_i);
  int32_t* dix = (int32_t*)(dd + b_desc + 2 * b_i);
  uint32_t* dwd = (uint32_t*)(dd + b_desc + 3 * b_i);
  double* dwt = (double*)(dd + b_desc + 4 * b_i);
  int32_t* dcounts = (int32_t*)(dd + b_desc + 4 * b_i + b_d);  // [0] = n_nodes, [1] = n_words
  ORBFE_HIP_CHECK(hipMemcpyAsync(dd, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
  const int st = launch_vocab(v, 1, dd, 0, nullptr, n, levelsup, bow ? dwd : nullptr, bow ? dwt : nullptr,
                              bow ? dcounts + 1 : nullptr, did, doff, dix, dcounts, n, v->stream);
  if (st) return st;
  int32_t cn[2] = {0, 0};
  ORBFE_HIP_CHECK(hipMemcpyAsync(cn, dcounts, 8, hipMemcpyDeviceToHost, v->stream));
  ORBFE_HIP_CHECK(hipStreamSynchronize(v->stream));
  const int nn = cn[0];
  ORBFE_HIP_CHECK(hipMemcpy(node_ids, did, 4 * (size_t)nn, hipMemcpyDeviceToHost));
  ORBFE_HIP_CHECK(hipMemcpy(offsets, doff, 4 * (size_t)(nn + 1), hipMemcpyDeviceToHost));
  const int total = offsets[nn];
  if (total > 0) ORBFE_HIP_CHECK(hipMemcpy(indices, dix, 4 * (size_t)total, hipMemcpyDeviceToHost));
  *n_nodes = nn;
  if (bow) {
    const int nw = cn[1];
    if (nw > 0) {
      ORBFE_HIP_CHECK(hipMemcpy(bow_words, dwd, 4 * (size_t)nw, hipMemcpyDeviceToHost));
      ORBFE_HIP_CHECK(hipMemcpy(bow_weights, dwt, 8 * (size_t)nw, hipMemcpyDeviceToHost));
    }
    *n_words = nw;
  }
  return ORBFE_OK;
}
