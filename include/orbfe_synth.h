/*
 * orbfe_synth.h -- seeded synthetic input frames (host code in liborbfe.so).
 *
 * Stands in for the KITTI 00 stereo PNGs the reference benchmarks on (absent offline); see
 * SURVEY.md section 8(d). Not part of the ORBextractor/ORBmatcher boundary.
 */
#ifndef ORBFE_SYNTH_H
#define ORBFE_SYNTH_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ORBFE_SYNTH_DEFAULT_RECTS 1200

/* Render stereo frame `index` (seed 0x0B5EED00 ^ index) at rows x cols into left and/or right
 * (either may be NULL), rows `step` bytes apart. n_rects <= 0 selects the default. */
int orbfe_synth_frame(uint64_t index, int rows, int cols, int n_rects, uint8_t* left,
                      uint8_t* right, size_t step);

/* Frame t of a seeded driving sequence (SURVEY 8(d), C3 KeyFrame pairs): a world of textured
 * billboards seen by a pinhole camera (fx, fy, cx, cy) at (0, 0, t * step_z) looking down +z, the
 * right camera `baseline` metres to the right (true stereo disparity fx * baseline / depth). Pose of
 * left frame t: Rcw = I, tcw = (0, 0, -t * step_z). Consecutive frames share most billboards, and
 * their epipole is (cx, cy). left and/or right (either may be NULL), rows `step` bytes apart. */
int orbfe_synth_sequence_frame(uint64_t seq_seed, long long t, int rows, int cols, float fx, float fy,
                               float cx, float cy, float baseline, float step_z, uint8_t* left,
                               uint8_t* right, size_t step);

#ifdef __cplusplus
}
#endif
#endif
