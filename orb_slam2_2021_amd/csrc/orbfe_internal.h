// orbfe_internal.h -- library-internal view of an extractor handle for the stereo stage
// (orbfe_stereo.hip). Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

#include "../../include/orbfe.h"

#define ORBFE_MAX_LEVELS 32

// The device pyramid (mvImagePyramid of every image) of the last extract call on a handle.
struct OrbfePyramid {
  const uint8_t* base;      // image i, level l: base + i*image_stride + off[l], rows pitch[l] apart
  long long image_stride;
  int n_images, nlevels;
  int w[ORBFE_MAX_LEVELS], h[ORBFE_MAX_LEVELS], pitch[ORBFE_MAX_LEVELS];
  long long off[ORBFE_MAX_LEVELS];
  float scale[ORBFE_MAX_LEVELS], inv_scale[ORBFE_MAX_LEVELS];
  int total_key_slots;      // orbfe_max_keypoints of the current geometry
  // device outputs of the last host-buffer extract call (stride total_key_slots per image)
  const orbfe_keypoint* io_kps;
  const uint8_t* io_desc;
  const int32_t* io_counts;
  hipStream_t stream;       // the handle's stream
  int device;
};

int orbfe_internal_pyramid(orbfe_extractor* h, OrbfePyramid* out);

// orbfe_extract_batch with a hook run right after the extraction's launches, before its results are
// copied down (calls of fewer than 8 images: the handle's stream, where the hook enqueues its own
// work and copies; the call's final wait covers them). An empty hook: orbfe_extract_batch.
// kps_img / desc_img (optional, n pointers each): image i's keypoints / descriptors go to
// kps_img[i] / desc_img[i] instead of kps + i * cap / desc + i * cap * 32.
int orbfe_internal_extract_batch(orbfe_extractor* h, int n, const uint8_t* const* imgs, int rows, int cols,
                                 size_t step, orbfe_keypoint* kps, uint8_t* desc, int cap, int32_t* counts,
                                 const std::function<int()>& after_launch, orbfe_keypoint* const* kps_img = nullptr,
                                 uint8_t* const* desc_img = nullptr);

// Stereo scratch owned by the handle (created lazily by orbfe_stereo.hip, freed with the handle).
struct OrbfeStereoScratch;
OrbfeStereoScratch** orbfe_internal_stereo_slot(orbfe_extractor* h);
void orbfe_internal_stereo_free(OrbfeStereoScratch* s);
