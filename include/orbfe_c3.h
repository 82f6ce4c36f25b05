/*
 * orbfe_c3.h -- one sub-batch of the C3 chain enqueued by one call (host code in liborbfe.so).
 *
 * The C3 step (BASELINE.json configs[2]) per sub-batch of B stereo frames:
 *   the stereo Frames' extraction (ORBextractor::operator() on 2B images, Frame.cc:113-116)
 *   + Frame::ComputeStereoMatches (Frame.cc:125), KeyFrame::ComputeBoW of the KeyFrame images
 *   (KeyFrame.cc:59-68), ORBmatcher::SearchForTriangulation of each KeyFrame pair
 *   (LocalMapping.cc:211-272).
 * orbfe_c3_run enqueues all of it -- the cross-stream waits, the extraction on a handle's stream,
 * the stereo stage, the vocabulary transform and the SearchForTriangulation batch on the matching
 * stream, and the ordering events -- in one call, instead of the ~25 separate C calls (and their
 * Python ctypes round trips) of orb_slam2_2021_amd/pipeline.py's per-stage path. Nothing blocks:
 * every result stays in the caller's device buffers.
 *
 * Buffers and handles belong to the caller and must outlive the plan. Streams / events are
 * hipStream_t / hipEvent_t passed as void* (orbfe_event_create events).
 */
#ifndef ORBFE_C3_H
#define ORBFE_C3_H
#include <stddef.h>
#include <stdint.h>

#include "orbfe.h"
#include "orbfe_match_batch.h"
#include "orbfe_vocab.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbfe_c3 orbfe_c3;

/* One output set (device pointers): image i's keypoints at kps + i*cap, descriptors at
 * desc + i*cap*32, count at counts[i]; the vocabulary's outputs per KeyFrame image with the
 * strides of orbfe_vocab_transform_batch_device (bow_* may be NULL: FeatureVector only); the
 * stereo outputs per pair p at u_right / depth + p*cap (NULL without stereo); the set's matcher
 * and its SearchForTriangulation pair descriptors (host array of n_pairs, copied at creation). */
typedef struct orbfe_c3_set {
  orbfe_keypoint* kps;
  uint8_t* desc;
  int32_t* counts;
  uint32_t* fv_node_ids;
  int32_t* fv_offsets;
  int32_t* fv_indices;
  int32_t* fv_n_nodes;
  uint32_t* bow_words;
  double* bow_weights;
  int32_t* bow_n;
  float* u_right;
  float* depth;
  orbfe_matcher* matcher;
  const orbfe_sft_pair* pairs;
} orbfe_c3_set;

typedef struct orbfe_c3_config {
  int n_images;         /* images per sub-batch (2B: the B lefts, then the B rights) */
  int rows, cols;       /* image shape; images pitch = cols, image_stride = rows * cols */
  int cap;              /* keypoint slots per image (>= orbfe_max_keypoints) */
  int n_vocab;          /* images 0..n_vocab-1 get a BowVector / FeatureVector */
  int levelsup;         /* KeyFrame::ComputeBoW's 4 */
  int n_stereo;         /* ComputeStereoMatches pairs (left p, right n_stereo + p); 0: none */
  float mbf, mb;        /* Frame::mbf, mb (orbfe_stereo.h) */
  int stereo_on_match;  /* ComputeStereoMatches on the matching stream (the handle's next
                           extraction waits for it) instead of right after the extraction */
  int n_pairs;          /* SearchForTriangulation pairs per set */
} orbfe_c3_config;

/* exts[n_exts]: extractor handles (handle k extracts on extract_streams[k % n_streams]);
 * match_stream: the vocabulary + matching stream, NULL to run them on each sub-batch's extraction
 * stream; sets[n_sets]: output sets (a set is reused only after its previous matching). */
int orbfe_c3_create(const orbfe_c3_config* cfg, orbfe_extractor* const* exts, int n_exts,
                    void* const* extract_streams, int n_streams, void* match_stream,
                    orbfe_vocabulary* voc, const orbfe_c3_set* sets, int n_sets, orbfe_c3** out);

/* Enqueue one sub-batch: n_images images at d_imgs (row pitch cols, image stride rows * cols)
 * into set `set` with handle `handle`. input_ready: an event the extraction waits for first (the
 * images' H2D copy), or NULL. defer_matched != 0: the set's "matched" event is not recorded; the
 * caller enqueues its own work on the matching stream (the C4 pack + gather) and then calls
 * orbfe_c3_finish. Returns ORBFE_OK or a negative ORBFE_ERR_*. */
int orbfe_c3_run(orbfe_c3* c, int set, int handle, const uint8_t* d_imgs, void* input_ready,
                 int defer_matched);

/* Record set `set`'s "matched" event on the stream its matching ran on; released: an event that
 * must also complete before the set is reused (work on another stream still reading it), or NULL. */
int orbfe_c3_finish(orbfe_c3* c, int set, void* released);

/* The stream set `set`'s last matching ran on (hipStream_t as void*). */
void* orbfe_c3_match_stream(orbfe_c3* c, int set);

int orbfe_c3_destroy(orbfe_c3* c);

#ifdef __cplusplus
}
#endif
#endif
