/*
 * orbfe_pack.h -- packing a device batch's used keypoint / descriptor slots for a variable-size
 * transfer (liborbfe.so). Used by the multi-GPU gather of BASELINE config C4: each rank sends rank 0
 * only the keypoints and descriptors it produced (the per-frame vectors ORBextractor::operator()
 * returns, ORBextractor.cc:1041-1103), not its fixed-capacity buffers.
 *
 * Packed layout (little endian): int32 n_images, int32 counts[n_images], zero padding to 16 B;
 * orbfe_keypoint kps[sum(counts)] (images in order), zero padding to 16 B; uint8 desc[sum][32].
 */
#ifndef ORBFE_PACK_H
#define ORBFE_PACK_H
#include <stddef.h>
#include <stdint.h>
#include "orbfe.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Bytes the packed form of `total_keypoints` keypoints over n_images needs. */
size_t orbfe_packed_bytes(int n_images, long long total_keypoints);

/* Device batch (image i: d_counts[i] keypoints at d_kps + i*cap, descriptors at d_desc + i*cap*32)
 * -> d_out (out_cap bytes; sized for the worst case orbfe_packed_bytes(n_images, n_images*cap)).
 * The packed size is written to *d_total_bytes (device int64). Async on `stream`. */
int orbfe_pack_keypoints_device(int n_images, const int32_t* d_counts, const orbfe_keypoint* d_kps,
                                const uint8_t* d_desc, int cap, uint8_t* d_out, size_t out_cap,
                                int64_t* d_total_bytes, void* stream);
#ifdef __cplusplus
}
#endif
#endif
