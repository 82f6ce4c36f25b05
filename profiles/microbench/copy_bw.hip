// Microbenchmark: how fast can byte-granular image rows be copied on MI355X (gfx950)?
// 64 images of 1241x376 (pitch 1241, as the bench's input) -> 64-byte aligned pitch 1280.
// build: hipcc --offload-arch=gfx950 -O3 -o copy_bw copy_bw.hip ; run: ./copy_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int W = 1241, H = 376, N = 64, P = 1280;

__global__ void byte4(const uint8_t* in, uint8_t* out) {  // k_copy0's pattern
  const int x = (blockIdx.x * 64 + threadIdx.x) * 4, y = blockIdx.y * 4 + threadIdx.y, img = blockIdx.z;
  if (x >= W || y >= H) return;
  const uint8_t* s = in + (size_t)img * W * H + (size_t)y * W + x;
  uint32_t v = 0;
  const int n = min(4, W - x);
  for (int k = 0; k < n; k++) v |= (uint32_t)s[k] << (8 * k);
  *reinterpret_cast<uint32_t*>(out + (size_t)img * P * H + (size_t)y * P + x) = v;
}

__global__ void byte16(const uint8_t* in, uint8_t* out) {  // 16 px per thread, byte loads
  const int x = (blockIdx.x * 64 + threadIdx.x) * 16, y = blockIdx.y * 4 + threadIdx.y, img = blockIdx.z;
  if (x >= W || y >= H) return;
  const uint8_t* s = in + (size_t)img * W * H + (size_t)y * W + x;
  uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 16; k++) if (x + k < W) v[k >> 2] |= (uint32_t)s[k] << (8 * (k & 3));
  uint4* d = reinterpret_cast<uint4*>(out + (size_t)img * P * H + (size_t)y * P + x);
  *d = make_uint4(v[0], v[1], v[2], v[3]);
}

__global__ void align16(const uint8_t* in, uint8_t* out) {  // aligned dwordx4 loads + alignbyte
  const int x = (blockIdx.x * 64 + threadIdx.x) * 16, y = blockIdx.y * 4 + threadIdx.y, img = blockIdx.z;
  if (x >= W || y >= H) return;
  const size_t off = (size_t)img * W * H + (size_t)y * W + x;
  const size_t a = off & ~(size_t)3;
  const int sh = (int)(off - a);
  const uint32_t* s = reinterpret_cast<const uint32_t*>(in + a);
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 5; k++) w[k] = s[k];  // may read 3 bytes past the row: inside the buffer here
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
  uint4* d = reinterpret_cast<uint4*>(out + (size_t)img * P * H + (size_t)y * P + x);
  *d = make_uint4(v[0], v[1], v[2], v[3]);
}

__global__ void vec16(const uint8_t* in, uint8_t* out) {  // aligned source (pitch P), 16 B / lane
  const int x = (blockIdx.x * 64 + threadIdx.x) * 16, y = blockIdx.y * 4 + threadIdx.y, img = blockIdx.z;
  if (x >= P || y >= H) return;
  const uint4 v = *reinterpret_cast<const uint4*>(in + (size_t)img * P * H + (size_t)y * P + x);
  *reinterpret_cast<uint4*>(out + (size_t)img * P * H + (size_t)y * P + x) = v;
}

template <typename K>
float run(K k, dim3 grid, dim3 block, const uint8_t* in, uint8_t* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k, grid, block, 0, 0, in, out);
  hipEventRecord(e0);
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(k, grid, block, 0, 0, in, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 20 * 1000;
}

int main() {
  uint8_t *in, *out;
  hipMalloc(&in, (size_t)N * P * H + 64);
  hipMalloc(&out, (size_t)N * P * H + 64);
  hipMemset(in, 7, (size_t)N * P * H);
  const double bytes = 2.0 * N * W * H;
  float t;
  t = run(byte4, dim3((W + 255) / 256, (H + 3) / 4, N), dim3(64, 4), in, out);
  printf("byte4   %7.1f us  %6.2f TB/s\n", t, bytes / t / 1e6);
  t = run(byte16, dim3((W + 1023) / 1024, (H + 3) / 4, N), dim3(64, 4), in, out);
  printf("byte16  %7.1f us  %6.2f TB/s\n", t, bytes / t / 1e6);
  t = run(align16, dim3((W + 1023) / 1024, (H + 3) / 4, N), dim3(64, 4), in, out);
  printf("align16 %7.1f us  %6.2f TB/s\n", t, bytes / t / 1e6);
  t = run(vec16, dim3((P + 1023) / 1024, (H + 3) / 4, N), dim3(64, 4), in, out);
  printf("vec16   %7.1f us  %6.2f TB/s (pitch-aligned source)\n", t, 2.0 * N * P * H / t / 1e6);
  return 0;
}
