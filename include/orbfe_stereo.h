/*
 * orbfe_stereo.h -- stereo matching of rectified pairs on the GPU (liborbfe.so, gfx950).
 *
 * Replaces, in the reference (lreithmayr/ORB_SLAM2_2021):
 *   Frame::ComputeStereoMatches()          src/Frame.cc:522-700 (declared include/Frame.h)
 *   the stereo Frame constructor's hot path src/Frame.cc:80-125 (ExtractORB(0/1) in two threads,
 *                                          then ComputeStereoMatches)
 *
 * Output per left keypoint i: u_right[i] (mvuRight) and depth[i] (mvDepth), -1 when unmatched,
 * bit-identical to the reference (the SAD search, parabola fit and median filter are restated
 * exactly; see DESIGN.md "ComputeStereoMatches").
 *
 * mb: the reference reads the member mb inside ComputeStereoMatches (Frame.cc:552) but assigns it
 * only afterwards (Frame.cc:149), so its maxD = mbf/mb uses whatever mb held. Callers pass the mb
 * they mean: mbf/fx for the documented behaviour, 0 for maxD = +inf (no near-range bound).
 */
#ifndef ORBFE_STEREO_H
#define ORBFE_STEREO_H
#include <stddef.h>
#include <stdint.h>

#include "orbfe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* n_pairs ComputeStereoMatches calls over images of the last orbfe_extract_batch_device call on h
 * (all pyramids still resident): pair p = left image left0 + p, right image right0 + p.
 * d_kps / d_desc / d_counts / cap are that call's outputs (image i at d_kps + i*cap, ...).
 * Writes d_u_right / d_depth at p*cap + i for i < d_counts[left0 + p]. Async on `stream`
 * (NULL: the handle's stream). Returns ORBFE_OK or a negative ORBFE_ERR_*. */
int orbfe_compute_stereo_matches_batch_device(orbfe_extractor* h, int n_pairs, int left0,
                                              int right0, const orbfe_keypoint* d_kps,
                                              const uint8_t* d_desc, const int32_t* d_counts,
                                              int cap, float mbf, float mb, float* d_u_right,
                                              float* d_depth, void* stream);

/* Host-buffer stereo frame (Frame.cc:113-125): extracts left and right in one batch, then
 * ComputeStereoMatches. The keypoint / descriptor outputs hold cap entries
 * (cap >= orbfe_max_keypoints(h, rows, cols)); u_right / depth hold cap floats. Blocking. On ORBFE_ERR_CAPACITY *n_l / *n_r hold the counts. */
int orbfe_stereo_frame(orbfe_extractor* h, const uint8_t* left, const uint8_t* right, int rows,
                       int cols, size_t step, float mbf, float mb, orbfe_keypoint* kps_l,
                       uint8_t* desc_l, int* n_l, orbfe_keypoint* kps_r, uint8_t* desc_r, int* n_r,
                       int cap, float* u_right, float* depth);

/* Host-buffer ComputeStereoMatches = the drop-in for Frame::ComputeStereoMatches with the
 * reference's two extractors (mpORBextractorLeft / mpORBextractorRight, Frame.cc:529,620-640):
 * the left pyramid is image `image_left` of h_left's last extract call, the right pyramid image
 * `image_right` of h_right's (h_left == h_right with images 0 / 1 after a two-image batch also
 * works). kps_* / desc_* are mvKeys / mDescriptors and mvKeysRight / mDescriptorsRight
 * (orbfe_keypoint has cv::KeyPoint's layout). Writes u_right / depth [n_l]. Blocking. */
int orbfe_compute_stereo_matches(orbfe_extractor* h_left, int image_left, orbfe_extractor* h_right,
                                 int image_right, const orbfe_keypoint* kps_l,
                                 const uint8_t* desc_l, int n_l, const orbfe_keypoint* kps_r,
                                 const uint8_t* desc_r, int n_r, float mbf, float mb,
                                 float* u_right, float* depth);

#ifdef __cplusplus
}
#endif
#endif
