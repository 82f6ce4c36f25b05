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
/* DistributeOctTree in two launches for device-resident batches (orbfe_extract_batch_device) of 8 or
 * more images: levels 0..k-1 with the full LDS
 * plan (80 KiB per block), levels k..L-1 with half of it (their smaller node arenas and key counts
 * fit 40 KiB: four blocks per CU); k <= 0 or k >= L: one launch of every level at 80 KiB. Default 5;
 * smaller batches and the host-buffer calls always take one launch (lower latency alone). */
int orbfe_debug_set_octree_split(orbfe_extractor* h, int k);
/* Latency schedule for calls of fewer than 8 images: FAST of levels 0..k-1 and their
 * DistributeOctTree on the handle's side stream while the main stream builds and processes levels
 * k..L-1; joined before the descriptors. Default k = 1; k <= 0 or k >= L: the throughput schedule
 * (FAST of the first levels on the side stream, one octree launch after every level's FAST). */
int orbfe_debug_set_latency_schedule(orbfe_extractor* h, int k);
/* DistributeOctTree's block size (256, 512 or 1024 threads; same results) for calls of fewer than 8
 * images (default 512) and for batches of 8+ (default 256). */
int orbfe_debug_set_octree_threads(orbfe_extractor* h, int small_calls, int batches);
/* Calls of fewer than 8 images: the block size of the octree launch that holds level 0 (the latency
 * schedule's side launch); 0 (default): the small calls' size. */
int orbfe_debug_set_octree_threads_l0(orbfe_extractor* h, int threads);
/* DistributeOctTree's node splits: a node of at most this many keys is split by one thread, a larger
 * one by a wavefront (1..128; default 48 for both), for calls of fewer than 8 images / batches. Same
 * results. */
int orbfe_debug_set_octree_serial(orbfe_extractor* h, int small_calls, int batches);
/* ComputePyramid's levels 1..L-1 in one k_pyramid launch of tx x ty tiles per image (each
 * workgroup builds its tile of every level, the previous level in LDS, the halo recomputed) for
 * calls of fewer than 8 images (default 16 x 12) / batches of 8+ (default 0 x 0: one k_resize_win
 * launch per level). Same bytes either way; a tiling whose tile needs more than 64 KiB of LDS falls
 * back to the chain. */
int orbfe_debug_set_pyramid_tiles(orbfe_extractor* h, int small_tx, int small_ty, int batch_tx, int batch_ty);
/* Calls of fewer than 8 images pick, per image count, between the latency schedule on the handle's two
 * streams and the same launch sequence on its launch stream alone by timing their first host-buffer
 * calls (4 warm-up, then 6 of each, alternating; one stream only if its mean, the largest sample
 * of each side dropped, is < 0.9x): the
 * runtime may have put both streams on one hardware queue, where cross-stream waits are slow.
 * enable = 0 (or ORBFE_SCHED_AUTOTUNE=0): always two streams. Resets the timings. */
int orbfe_debug_set_schedule_autotune(orbfe_extractor* h, int enable);
/* Batches: FAST of the side-stream levels 1..k-1 (orbfe_debug_set_fast_side_levels) in one launch
 * once level k-1 is built, instead of one launch (and event pair) per level as each is built. */
int orbfe_debug_set_fast_side_merge(orbfe_extractor* h, int merge);
/* The autotune's choice for calls of n_images (1..7) images: -1 still timing, 0 two streams, 1 one. */
int orbfe_debug_schedule_choice(const orbfe_extractor* h, int n_images);
/* Host-buffer calls of fewer than 8 images: k_copy0 reads the staged image straight from pinned host
 * memory (input != 0, the default) instead of after a separate H2D copy, and (output != 0, the
 * default; calls without a device-side consumer of the outputs) the kernels write the results into
 * the pinned host mirror instead of a device block copied down afterwards. input = 2 stages the
 * image in the level-0 layout instead (padded rows, REFLECT_101 columns written by the host; one
 * straight k_copy_l0 copy): not faster. Same results. */
int orbfe_debug_set_zero_copy(orbfe_extractor* h, int input, int output);
/* The LDS budgets (KiB per block) of the two octree launches: levels below the split (default 80)
 * and from it on (default 40). Keys beyond a plan's capacity take the global-memory path. */
int orbfe_debug_set_octree_lds(orbfe_extractor* h, int hi_kb, int lo_kb);
/* k_fast cells (wavefronts) per workgroup: the side-stream launches of the early levels (default 4)
 * and the launch of the remaining levels (default 1); 1, 2, 4 or 8. */
int orbfe_debug_set_fast_wpb(orbfe_extractor* h, int side_wpb, int main_wpb);
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
/* Launch-graph counters of the handle: captures, replays, graphs held (3 values). */
int orbfe_debug_graph_stats(const orbfe_extractor* h, long long* out3);
/* The IC_Angle circle's row extents umax[0..15] the handle computed (ORBextractor.cc:457-472). */
int orbfe_debug_get_umax(const orbfe_extractor* h, int32_t* umax16);
/* computeOrbDescriptor's steering cos / sin (ORBextractor.cc:109-110) exactly as k_describe
 * computes them (a port of glibc's cosf / sinf), for the float degree values with bit patterns
 * deg_bits_begin .. deg_bits_begin + n - 1, into device buffers (NULL stream = default stream;
 * synchronous). Used by the exhaustive glibc check, tests/test_gpu_trig.py. */
int orbfe_debug_steer_trig(uint32_t deg_bits_begin, uint32_t n, float* d_cos, float* d_sin, void* stream);
/* The last SearchByProjection's k_sbp_sweep statistics (the claim order after round 0, one
 * workgroup, chunk by chunk): [0] chunks, [1] Jacobi rounds summed over chunks, [2] live queries
 * (round 0 pruned the rest), [3] chunks finished by the sequential walk, [4] the most rounds one
 * chunk took; wall-clock ticks (100 MHz) in [5] the compaction of the live queries, [6] the chunks'
 * loads, [7] their rounds, [8] their commits; [9] live queries past the cache (grid walk each
 * round); [10] shader clock cycles / 1000 and [11] 100 MHz ticks over the kernel (its clock rate). */
int orbfe_debug_matcher_sweep_stats(orbfe_matcher* m, int32_t* out12);
/* Test knobs of the sweep for this matcher (0: the default): live queries per chunk (1 .. 1024;
 * small chunks commit claims across many chunks), Jacobi rounds a chunk may take before the
 * reference's sequential loop over it (1 forces that walk), candidate-cache entries per query (48;
 * small values send queries past the cache to the grid walk). */
int orbfe_debug_matcher_set_sweep(orbfe_matcher* m, int chunk, int max_rounds, int cand_cap);

#ifdef __cplusplus
}
#endif
#endif
