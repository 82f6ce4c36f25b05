/*
 * orbfe_match_batch.h -- device-resident batch entry points of the matcher (liborbfe.so).
 *
 * For pipelines whose keypoints, descriptors and feature vectors already live in HBM (the
 * benchmark's extract -> SearchForTriangulation step). All pointers inside the structs are DEVICE
 * pointers; the struct arrays themselves are host memory and are copied on every call.
 */
#ifndef ORBFE_MATCH_BATCH_H
#define ORBFE_MATCH_BATCH_H
#include <stdint.h>
#include "orbfe.h"
#ifdef __cplusplus
extern "C" {
#endif

/* One SearchForTriangulation(KF1, KF2, F12, pairs, bOnlyStereo) call (ORBmatcher.cc:671-839). */
typedef struct orbfe_sft_pair {
  orbfe_frame_view kf1, kf2;
  orbfe_feature_vector fv1, fv2;
  float f12[9];
  float ex, ey;
  int32_t* match12;   /* out: kf1.n entries */
  int32_t* nmatches;  /* out: 1 entry */
  /* Optional device-side sizes, for inputs produced on the device in the same stream (NULL =
   * use kf1.n / kf2.n / fv1.n_nodes / fv2.n_nodes). With fv1_nodes_dev set, fv1.n_nodes must
   * still hold an upper bound of the node count: it sizes the launch grid. */
  const int32_t* kf1_n_dev;
  const int32_t* kf2_n_dev;
  const int32_t* fv1_nodes_dev;
  const int32_t* fv2_nodes_dev;
} orbfe_sft_pair;

/* n_pairs independent SearchForTriangulation calls, async on `stream` (NULL = the matcher's
 * stream). */
int orbfe_search_for_triangulation_batch_device(orbfe_matcher* m, int n_pairs,
                                                const orbfe_sft_pair* pairs, int only_stereo,
                                                void* stream);

/* hipStream_t of the matcher (as void*). */
void* orbfe_matcher_stream(orbfe_matcher* m);
/* Profiling of the host-buffer searches (SearchByProjection family, isInFrustum + SearchLocalPoints):
 * with it on, each call records HIP events around its device part (first kernel to last kernel,
 * H2D / D2H excluded); orbfe_matcher_last_device_ms returns the last call's device milliseconds. */
int orbfe_matcher_set_profiling(orbfe_matcher* m, int on);
int orbfe_matcher_last_device_ms(orbfe_matcher* m, float* ms);

/* Statistics of the last SearchByProjection call: fixpoint rounds run and whether the serial
 * fallback kernel had to finish the claim order. */
int orbfe_matcher_last_stats(orbfe_matcher* m, int* rounds, int* serial_used);

/* The SearchByProjection claim-order fixpoint runs 12 rounds in its first launch; a host-buffer
 * search whose fixpoint has not settled then continues in doubling chunks (up to 1024 rounds)
 * before the serial kernel would finish the claim order. This call fixes the budget to `rounds`
 * (1..12) with no continuation, so that the serial kernel runs past it; tests use it to exercise
 * that path. */
int orbfe_matcher_set_max_rounds(orbfe_matcher* m, int rounds);

#ifdef __cplusplus
}
#endif
#endif
