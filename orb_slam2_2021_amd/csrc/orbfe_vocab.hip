// orbfe_vocab.hip -- DBoW2 vocabulary descent to FeatureVector CSR on gfx950.
//
// Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1140-1207 (transform of a descriptor
// set into BowVector + FeatureVector) and :1231-1272 (descent of one descriptor: at every level the
// child with the smallest FORB::distance, strict '<' so the first best wins; the node reached at
// level L - levelsup is the FeatureVector node; a word whose weight is 0 is skipped). KeyFrame::
// ComputeBoW (KeyFrame.cc:59-68) calls it with levelsup = 4; SearchForTriangulation consumes the
// FeatureVector (ORBmatcher.cc:674-804).
//
// One workgroup per image: every thread descends its descriptors (children contiguous in BFS
// order, centroids read through L2), then the (node, feature) keys are sorted stably in LDS with a
// bitonic network and split into CSR -- node ids ascending, features ascending inside a node,
// exactly the std::map<NodeId, vector<unsigned>> iteration order.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_vocab.h"
#include "orbfe_device.h"

#define VOCAB_MAX_FEATURES 8192

struct orbfe_vocabulary {
  int device = 0;
  int n_nodes = 0, levels = 0;
  uint8_t* d_desc = nullptr;
  int32_t* d_first = nullptr;
  int32_t* d_nchild = nullptr;
  float* d_weight = nullptr;
  hipStream_t stream = nullptr;
  // host-call scratch
  uint8_t* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  unsigned long long* d_keys = nullptr;  // (node, feature) keys between the two kernels
  size_t keys_bytes = 0;
};

struct VocabArgs {
  const uint8_t* vdesc;
  const int32_t* first;
  const int32_t* nchild;
  const float* weight;
  int nid_level;
  const uint8_t* desc;
  long long desc_stride;  // bytes between images
  const int32_t* counts;  // per image feature count (device)
  int fixed_count;        // used when counts == NULL
  uint32_t* node_ids;
  int32_t* offsets;
  int32_t* indices;
  int32_t* n_nodes;
  int cap;                // per-image capacity of node_ids / indices; offsets hold cap + 1
};

// k_vocab_descend: one thread per descriptor of every image (TemplatedVocabulary.h:1231-1272);
// writes the (node, feature) key, or ~0 for a stopped word / an empty slot.
__global__ __launch_bounds__(256) void k_vocab_descend(VocabArgs a, unsigned long long* keys) {
  const int img = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.cap) return;
  const int n = min(a.counts ? a.counts[img] : a.fixed_count, a.cap);
  unsigned long long key = ~0ull;
  if (i < n) {
    const uint8_t* desc = a.desc + (long long)img * a.desc_stride;
    uint4 d0, d1;
    load_desc(desc + (size_t)i * 32, d0, d1);
    int node = 0, level = 0, nid = 0;
    while (a.nchild[node] > 0) {
      ++level;
      const int f = a.first[node], nc = a.nchild[node];
      int best = f, best_d;
      {
        uint4 c0, c1;
        load_desc(a.vdesc + (size_t)f * 32, c0, c1);
        best_d = hamming256(d0, d1, c0, c1);
      }
      for (int c = 1; c < nc; c++) {
        uint4 c0, c1;
        load_desc(a.vdesc + (size_t)(f + c) * 32, c0, c1);
        const int dd = hamming256(d0, d1, c0, c1);
        if (dd < best_d) {  // strict: the first best child wins
          best_d = dd;
          best = f + c;
        }
      }
      node = best;
      if (level == a.nid_level) nid = node;
    }
    if (a.weight[node] > 0) key = ((unsigned long long)(unsigned)nid << 32) | (unsigned)i;
  }
  keys[(long long)img * a.cap + i] = key;
}

// k_vocab_csr: one 1024-thread workgroup per image sorts its keys stably (bitonic in LDS) and
// emits CSR.
#define VOCAB_THREADS 1024
__global__ __launch_bounds__(VOCAB_THREADS) void k_vocab(VocabArgs a, const unsigned long long* keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long skeys[];
  __shared__ int s_n;
  const int img = blockIdx.x, t = threadIdx.x;
  const int n = min(a.counts ? a.counts[img] : a.fixed_count, a.cap);
  int P2 = 1;
  while (P2 < n) P2 <<= 1;
  for (int i = t; i < P2; i += VOCAB_THREADS) skeys[i] = i < n ? keys[(long long)img * a.cap + i] : ~0ull;
  __syncthreads();
  // bitonic sort, ascending; every thread owns P2/2048 compare-exchange pairs per stage
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
  // CSR: a node starts where its id differs from the previous key's. Each thread owns a
  // contiguous chunk of the sorted keys; starts are counted, scanned and written in order.
  __shared__ int s_wsum[VOCAB_THREADS / 64];
  uint32_t* ids = a.node_ids + (long long)img * a.cap;
  int32_t* offs = a.offsets + (long long)img * (a.cap + 1);
  int32_t* idx = a.indices + (long long)img * a.cap;
  if (t == 0) s_n = 0;
  __syncthreads();
  int nvalid = 0;
  for (int i = t; i < n; i += VOCAB_THREADS) nvalid += skeys[i] != ~0ull;
  nvalid = wave_sum(nvalid);
  if (lane_id() == 0) atomicAdd(&s_n, nvalid);
  __syncthreads();
  const int nv = s_n;  // valid keys sort first
  for (int i = t; i < nv; i += VOCAB_THREADS) idx[i] = (int32_t)(skeys[i] & 0xffffffffull);
  const int per = (nv + VOCAB_THREADS - 1) / VOCAB_THREADS;
  const int beg = min(t * per, nv), end = min(beg + per, nv);
  auto is_start = [&](int i) {
    return i == 0 || (uint32_t)(skeys[i] >> 32) != (uint32_t)(skeys[i - 1] >> 32);
  };
  int cnt = 0;
  for (int i = beg; i < end; i++) cnt += is_start(i);
  // exclusive scan of cnt over the workgroup
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
  int nodes = 0;
  for (int k = 0; k < VOCAB_THREADS / 64; k++) nodes += s_wsum[k];
  for (int i = beg; i < end; i++) {
    if (is_start(i)) {
      ids[pos] = (uint32_t)(skeys[i] >> 32);
      offs[pos] = i;
      pos++;
    }
  }
  if (t == 0) {
    offs[nodes] = nv;
    a.n_nodes[img] = nodes;
  }
}

extern "C" int orbfe_vocab_create(int n_nodes, int levels, const uint8_t* node_desc,
                                  const int32_t* first_child, const int32_t* n_children,
                                  const float* weights, int device, orbfe_vocabulary** out) {
  if (!out || n_nodes <= 0 || levels <= 0 || !node_desc || !first_child || !n_children || !weights)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_create: bad argument");
  *out = nullptr;
  for (int i = 0; i < n_nodes; i++)
    if (n_children[i] < 0 || (n_children[i] > 0 && (first_child[i] <= i || first_child[i] + n_children[i] > n_nodes)))
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_create: malformed tree");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return orbfe_set_error(ORBFE_ERR_HIP, "orbfe_vocab_create: no such HIP device");
  orbfe_vocabulary* v = new orbfe_vocabulary();
  v->device = device;
  v->n_nodes = n_nodes;
  v->levels = levels;
  auto fail = [&](hipError_t e, const char* w) {
    hipFree(v->d_desc);
    hipFree(v->d_first);
    hipFree(v->d_nchild);
    hipFree(v->d_weight);
    delete v;
    return orbfe_set_hip_error(e, w);
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail(e, "hipSetDevice");
  if ((e = hipMalloc(&v->d_desc, (size_t)n_nodes * 32)) != hipSuccess) return fail(e, "hipMalloc");
  if ((e = hipMalloc(&v->d_first, 4 * (size_t)n_nodes)) != hipSuccess) return fail(e, "hipMalloc");
  if ((e = hipMalloc(&v->d_nchild, 4 * (size_t)n_nodes)) != hipSuccess) return fail(e, "hipMalloc");
  if ((e = hipMalloc(&v->d_weight, 4 * (size_t)n_nodes)) != hipSuccess) return fail(e, "hipMalloc");
  hipMemcpy(v->d_desc, node_desc, (size_t)n_nodes * 32, hipMemcpyHostToDevice);
  hipMemcpy(v->d_first, first_child, 4 * (size_t)n_nodes, hipMemcpyHostToDevice);
  hipMemcpy(v->d_nchild, n_children, 4 * (size_t)n_nodes, hipMemcpyHostToDevice);
  if ((e = hipMemcpy(v->d_weight, weights, 4 * (size_t)n_nodes, hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "hipMemcpy");
  if ((e = hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(e, "hipStreamCreate");
  *out = v;
  return ORBFE_OK;
}

extern "C" int orbfe_vocab_destroy(orbfe_vocabulary* v) {
  if (!v) return ORBFE_OK;
  hipSetDevice(v->device);
  if (v->stream) hipStreamSynchronize(v->stream);
  hipFree(v->d_desc);
  hipFree(v->d_first);
  hipFree(v->d_nchild);
  hipFree(v->d_weight);
  hipFree(v->d_scratch);
  hipFree(v->d_keys);
  if (v->stream) hipStreamDestroy(v->stream);
  delete v;
  return ORBFE_OK;
}

static int launch_vocab(orbfe_vocabulary* v, int n_images, const uint8_t* d_desc,
                        size_t desc_stride, const int32_t* d_counts, int fixed_count, int levelsup,
                        uint32_t* d_node_ids, int32_t* d_offsets, int32_t* d_indices,
                        int32_t* d_n_nodes, int cap, hipStream_t s) {
  if (cap <= 0 || cap > VOCAB_MAX_FEATURES)
    return orbfe_set_error(ORBFE_ERR_ARG, "vocab transform: cap must be in 1..8192");
  VocabArgs a;
  a.vdesc = v->d_desc;
  a.first = v->d_first;
  a.nchild = v->d_nchild;
  a.weight = v->d_weight;
  a.nid_level = v->levels - levelsup;
  a.desc = d_desc;
  a.desc_stride = (long long)desc_stride;
  a.counts = d_counts;
  a.fixed_count = fixed_count;
  a.node_ids = d_node_ids;
  a.offsets = d_offsets;
  a.indices = d_indices;
  a.n_nodes = d_n_nodes;
  a.cap = cap;
  int P2 = 1;
  while (P2 < cap) P2 <<= 1;
  const size_t need = sizeof(unsigned long long) * (size_t)cap * n_images;
  if (need > v->keys_bytes) {
    hipFree(v->d_keys);
    v->d_keys = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&v->d_keys, need));
    v->keys_bytes = need;
  }
  hipLaunchKernelGGL(k_vocab_descend, dim3((cap + 255) / 256, n_images), dim3(256), 0, s, a, v->d_keys);
  hipLaunchKernelGGL(k_vocab, dim3(n_images), dim3(VOCAB_THREADS), sizeof(unsigned long long) * P2, s, a,
                     (const unsigned long long*)v->d_keys);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}

extern "C" int orbfe_vocab_transform_batch_device(orbfe_vocabulary* v, int n_images,
                                                  const uint8_t* d_desc, size_t desc_stride,
                                                  const int32_t* d_counts, int levelsup,
                                                  uint32_t* d_node_ids, int32_t* d_offsets,
                                                  int32_t* d_indices, int32_t* d_n_nodes, int cap,
                                                  void* stream) {
  if (!v || n_images < 0 || (n_images > 0 && (!d_desc || !d_counts || !d_node_ids || !d_offsets ||
                                              !d_indices || !d_n_nodes)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_transform_batch_device: bad argument");
  if (n_images == 0) return ORBFE_OK;
  hipSetDevice(v->device);
  return launch_vocab(v, n_images, d_desc, desc_stride, d_counts, 0, levelsup, d_node_ids,
                      d_offsets, d_indices, d_n_nodes, cap, stream ? (hipStream_t)stream : v->stream);
}

extern "C" int orbfe_vocab_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                                     uint32_t* node_ids, int32_t* offsets, int32_t* indices,
                                     int* n_nodes) {
  if (!v || n < 0 || !n_nodes || (n > 0 && (!desc || !node_ids || !offsets || !indices)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_vocab_transform: bad argument");
  if (n == 0) {
    *n_nodes = 0;
    if (offsets) offsets[0] = 0;
    return ORBFE_OK;
  }
  if (n > VOCAB_MAX_FEATURES) return orbfe_set_error(ORBFE_ERR_ARG, "too many descriptors");
  hipSetDevice(v->device);
  const size_t b_desc = ((size_t)n * 32 + 255) & ~(size_t)255, b_ids = ((size_t)n * 4 + 255) & ~(size_t)255;
  const size_t need = b_desc + 3 * b_ids + 512;
  if (need > v->scratch_bytes) {
    hipFree(v->d_scratch);
    v->d_scratch = nullptr;
    ORBFE_HIP_CHECK(hipMalloc(&v->d_scratch, need));
    v->scratch_bytes = need;
  }
  uint8_t* dd = v->d_scratch;
  uint32_t* did = (uint32_t*)(dd + b_desc);
  int32_t* doff = (int32_t*)(dd + b_desc + b_ids);
  int32_t* dix = (int32_t*)(dd + b_desc + 2 * b_ids + 256);
  int32_t* dnn = (int32_t*)(dd + b_desc + 3 * b_ids + 256);
  ORBFE_HIP_CHECK(hipMemcpyAsync(dd, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
  int st = launch_vocab(v, 1, dd, 0, nullptr, n, levelsup, did, doff, dix, dnn, n, v->stream);
  if (st) return st;
  int32_t nn = 0;
  ORBFE_HIP_CHECK(hipMemcpyAsync(&nn, dnn, 4, hipMemcpyDeviceToHost, v->stream));
  ORBFE_HIP_CHECK(hipStreamSynchronize(v->stream));
  ORBFE_HIP_CHECK(hipMemcpy(node_ids, did, 4 * (size_t)nn, hipMemcpyDeviceToHost));
  ORBFE_HIP_CHECK(hipMemcpy(offsets, doff, 4 * (size_t)(nn + 1), hipMemcpyDeviceToHost));
  int32_t total = 0;
  ORBFE_HIP_CHECK(hipMemcpy(&total, doff + nn, 4, hipMemcpyDeviceToHost));
  if (total > 0) ORBFE_HIP_CHECK(hipMemcpy(indices, dix, 4 * (size_t)total, hipMemcpyDeviceToHost));
  *n_nodes = nn;
  return ORBFE_OK;
}
