/*
 * orbfe_debug.h -- stage-inspection hooks of liborbfe.so used by the per-stage parity tests.
 * Not part of the ORBextractor/ORBmatcher boundary. Keys are packed x | y<<12 | score<<24.
 */
#ifndef ORBFE_DEBUG_H
#define ORBFE_DEBUG_H
#include <stdint.h>
#include "orbfe.h"
#ifdef __cplusplus
extern "C" {
#endif
/* FAST candidates of (image, level) of the last extract call, in DistributeOctTree input order,
 * coordinates relative to minBorder (16). */
int orbfe_debug_get_candidates(orbfe_extractor* h, int image, int level, uint32_t* out, int cap,
                               int* n);
/* FAST candidates of every image and level of the last extract call (one D2H of the cell counts). */
int orbfe_debug_candidate_total(orbfe_extractor* h, long long* total);
/* Octree survivors of (image, level) in output order, level coordinates. */
int orbfe_debug_get_level_keys(orbfe_extractor* h, int image, int level, uint32_t* out, int cap,
                               int* n);
/* GaussianBlur(7x7, 2, REFLECT_101) of (image, level) as computed for the descriptors. */
int orbfe_debug_get_blurred(orbfe_extractor* h, int image, int level, uint8_t* out, int cap);
/* Per level: w, h, ncells, candidate capacity, budget, nIni, key capacity (7 ints per level). */
int orbfe_debug_geometry(orbfe_extractor* h, int rows, int cols, int32_t* info, int cap);
/* Cap the per-level key count DistributeOctTree keeps in LDS (rounded down to 64; 0 forces the
 * global-memory path for every level; < 0 restores the automatic size). */
int orbfe_debug_set_octree_key_cap(orbfe_extractor* h, int cap);
/* FAST of levels 0..k-1 on the side stream, each launched as soon as its level is built, the rest
 * in one launch after the resize chain (k <= 0: the default, levels 0..2). */
int orbfe_debug_set_fast_side_levels(orbfe_extractor* h, int k);
/* 1: run the side-stream work (k_blur, the early FAST levels) on the launch stream, for callers
 * that overlap whole extractions on several streams of their own; 0 (default): the handle's
 * high-priority side stream. */
int orbfe_debug_set_inline_side(orbfe_extractor* h, int on);
/* The side-stream work on a caller's stream (e.g. one high-priority stream shared by several
 * handles whose extractions overlap); NULL restores the handle's own side stream. */
int orbfe_set_side_stream(orbfe_extractor* h, void* stream);
/* Where GaussianBlur runs: 0 (default) on the side stream beside DistributeOctTree, 1 on the
 * launch stream after DistributeOctTree (several handles sharing one side stream). */
int orbfe_debug_set_blur_mode(orbfe_extractor* h, int mode);
/* The IC_Angle circle's row extents umax[0..15] the handle computed (ORBextractor.cc:457-472). */
int orbfe_debug_get_umax(const orbfe_extractor* h, int32_t* umax16);
/* computeOrbDescriptor's steering cos / sin (ORBextractor.cc:109-110) exactly as k_describe
 * computes them (a port of glibc's cosf / sinf), for the float degree values with bit patterns
 * deg_bits_begin .. deg_bits_begin + n - 1, into device buffers (NULL stream = default stream;
 * synchronous). Used by the exhaustive glibc check, tests/test_gpu_trig.py. */
int orbfe_debug_steer_trig(uint32_t deg_bits_begin, uint32_t n, float* d_cos, float* d_sin, void* stream);
/* The last SearchByProjection's k_sbp_settle statistics: rounds that scanned every query (a
 * keypoint listed by more queries than the inverted index holds), queries re-evaluated, keypoint
 * owners recomputed (all summed over its rounds; zeros when the per-round launches ran), then the
 * kernel's wall-clock ticks (100 MHz) in its prologue and in its steps a-d, summed over rounds. */
int orbfe_debug_matcher_settle_stats(orbfe_matcher* m, int32_t* out8);
/* The first SearchByProjection round k_sbp_settle runs for this matcher (2 .. 12; 0 restores the
 * default, round 8): tests drive the settle kernel through most of the fixpoint with 2. */
int orbfe_debug_matcher_set_settle_from(orbfe_matcher* m, int round0);

#ifdef __cplusplus
}
#endif
#endif
