// orbfe_pack.hip -- pack the used keypoint / descriptor slots of a device batch (include/orbfe_pack.h)
// for the C4 gather: one workgroup per image finds its offset (sum of the earlier counts), copies
// its keypoints as dwords and its descriptors as 16-byte vectors; workgroup 0 also writes the
// header and the total size. HBM-bound copy of the used bytes only.
#include <hip/hip_runtime.h>

#include "../../include/orbfe.h"
#include "../../include/orbfe_pack.h"
#include "orbfe_device.h"
#include "orbfe_ktimer.h"

static __host__ __device__ inline long long align16(long long x) { return (x + 15) & ~15ll; }

extern "C" size_t orbfe_packed_bytes(int n_images, long long total_keypoints) {
  const long long head = align16(4 * (1 + (long long)n_images));
  return (size_t)(align16(head + 28 * total_keypoints) + 32 * total_keypoints);
}

__global__ __launch_bounds__(256) void k_pack(int n_images, const int32_t* __restrict__ counts,
                                              const orbfe_keypoint* __restrict__ kps,
                                              const uint8_t* __restrict__ desc, int cap,
                                              uint8_t* __restrict__ out, int64_t* total_bytes) {
  __shared__ long long s_part[4];
  const int img = blockIdx.x, t = threadIdx.x;
  long long before = 0, all = 0;
  for (int j = t; j < n_images; j += 256) {
    const long long c = min(max(counts[j], 0), cap);
    all += c;
    if (j < img) before += c;
  }
  // workgroup sums of (before, all): pack both into one 64-bit lane sum; the host check keeps
  // n_images * cap < 2^31, so neither 32-bit half can carry into the other
  unsigned long long v = ((unsigned long long)before << 32) | (unsigned long long)all;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane_id() == 0) s_part[wave_id()] = (long long)v;
  __syncthreads();
  v = (unsigned long long)(s_part[0] + s_part[1] + s_part[2] + s_part[3]);
  before = (long long)(v >> 32);
  all = (long long)(v & 0xffffffffull);
  const long long head = align16(4 * (1 + (long long)n_images));
  const long long desc_off = align16(head + 28 * all);
  const int n = min(max(counts[img], 0), cap);
  // keypoints: 7 dwords each
  const uint32_t* ksrc = reinterpret_cast<const uint32_t*>(kps + (size_t)img * cap);
  uint32_t* kdst = reinterpret_cast<uint32_t*>(out + head + 28 * before);
  for (int i = t; i < 7 * n; i += 256) kdst[i] = ksrc[i];
  const uint4* dsrc = reinterpret_cast<const uint4*>(desc + (size_t)img * cap * 32);
  uint4* ddst = reinterpret_cast<uint4*>(out + desc_off + 32 * before);
  for (int i = t; i < 2 * n; i += 256) ddst[i] = dsrc[i];
  if (img == 0) {
    int32_t* h = reinterpret_cast<int32_t*>(out);
    for (int j = t; j < n_images; j += 256) h[1 + j] = min(max(counts[j], 0), cap);
    if (t == 0) h[0] = n_images;
    for (long long p = 4 * (1 + (long long)n_images) + t; p < head; p += 256) out[p] = 0;
    for (long long p = head + 28 * all + t; p < desc_off; p += 256) out[p] = 0;
    if (t == 0) *total_bytes = desc_off + 32 * all;
  }
}

extern "C" int orbfe_pack_keypoints_device(int n_images, const int32_t* d_counts,
                                           const orbfe_keypoint* d_kps, const uint8_t* d_desc, int cap,
                                           uint8_t* d_out, size_t out_cap, int64_t* d_total_bytes,
                                           void* stream) {
  if (n_images <= 0 || cap <= 0 || !d_counts || !d_kps || !d_desc || !d_out || !d_total_bytes ||
      n_images > (1 << 20))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_pack_keypoints_device: bad argument");
  if ((long long)n_images * cap >= (1ll << 31))  // k_pack sums keypoint counts in 32-bit halves
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_pack_keypoints_device: n_images * cap must stay below 2^31");
  if (out_cap < orbfe_packed_bytes(n_images, (long long)n_images * cap))
    return orbfe_set_error(ORBFE_ERR_CAPACITY, "orbfe_pack_keypoints_device: out_cap below the worst case");
  ORBFE_LAUNCH("k_pack", k_pack, dim3(n_images), dim3(256), 0, (hipStream_t)stream, n_images, d_counts, d_kps,
                     d_desc, cap, d_out, d_total_bytes);
  ORBFE_HIP_CHECK(hipGetLastError());
  return ORBFE_OK;
}
