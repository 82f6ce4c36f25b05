/*
 * orbref.h -- C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a plain C++17 restatement of ORB-SLAM2's per-frame feature path
 * (src/ORBextractor.cc, src/ORBmatcher.cc, src/Frame.cc of lreithmayr/ORB_SLAM2_2021) with the
 * OpenCV 4.5.x primitives it calls (FAST, resize INTER_LINEAR, GaussianBlur, fastAtan2, cvRound)
 * re-specified from their published algorithms. It is only ever loaded by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, always as the checker -- never by
 * the product path (orb_slam2_2021_amd/).
 *
 * Parity status (see DESIGN.md "Oracle"): the ORB-SLAM2 tables (umax, per-level budgets, scale
 * tables, the 256-pair pattern, Gaussian taps) are pinned by known-answer tests; the reference
 * itself cannot be built here (it needs OpenCV/Boost/Eigen, none present), so results at the
 * OpenCV boundary are "parity unpinned".
 *
 * Matcher structs are the product's own boundary structs (include/orbfe.h).
 */
#ifndef ORBREF_H
#define ORBREF_H
#include <stddef.h>
#include <stdint.h>
#include "../include/orbfe.h"
#include "../include/orbfe_frustum.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbref_extractor orbref_extractor;

orbref_extractor* orbref_extractor_create(int nfeatures, float scale_factor, int nlevels,
                                          int ini_th, int min_th);
void orbref_extractor_destroy(orbref_extractor* h);
int orbref_set_resize_mode(orbref_extractor* h, int mode);
int orbref_get_tables(const orbref_extractor* h, float* scale, float* inv_scale, float* sigma2,
                      float* inv_sigma2, int32_t* features_per_level, int32_t* umax16);
int orbref_extract(orbref_extractor* h, const uint8_t* img, int rows, int cols, size_t step,
                   orbfe_keypoint* kps, int cap, uint8_t* desc, int* n);
/* Stage outputs of the last extract call (for per-stage parity). */
int orbref_get_level(const orbref_extractor* h, int level, uint8_t* out, int cap, int* rows,
                     int* cols);
/* FAST candidates of `level` in DistributeOctTree input order, packed x | y<<12 | score<<24
 * (coordinates relative to minBorder = 16). */
int orbref_get_candidates(const orbref_extractor* h, int level, uint32_t* out, int cap, int* n);
/* Octree survivors of `level` in output order, same packing, level coordinates. */
int orbref_get_level_keys(const orbref_extractor* h, int level, uint32_t* out, int cap, int* n);

/* Primitives. */
int orbref_resize_linear(const uint8_t* src, int sw, int sh, int sstep, uint8_t* dst, int dw,
                         int dh, int dstep, int mode);
int orbref_gaussian_blur7(const uint8_t* src, int w, int h, int sstep, uint8_t* dst, int dstep);
float orbref_fast_atan2(float y, float x);
int orbref_fast_score_map(const uint8_t* img, int w, int h, int step, uint8_t* m_out);
int orbref_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Matchers (host memory, same semantics and outputs as the orbfe_* functions). */
int orbref_search_by_projection_local(const orbfe_frame_view* frame,
                                      const orbfe_local_mappoints* mps, float th, float nnratio,
                                      int32_t* best_idx, int* nmatches);
int orbref_search_by_projection_lastframe(const orbfe_frame_view* current,
                                          const orbfe_lastframe_mappoints* last,
                                          const float* tcw_cur, float th, int mono,
                                          int check_ori, int32_t* best_idx, int* nmatches);
int orbref_search_for_triangulation(const orbfe_frame_view* kf1, const orbfe_frame_view* kf2,
                                    const orbfe_feature_vector* fv1,
                                    const orbfe_feature_vector* fv2, const float* f12, float ex,
                                    float ey, int only_stereo, int check_ori, int32_t* match12,
                                    int* nmatches);
/* The DBoW2 vocabulary (orbref_vocab.cpp): the reference's loaders and transform with its own
 * containers (std::map BowVector / FeatureVector, child-id vectors, double weights). */
typedef struct orbref_vocab orbref_vocab;
int orbref_vocab_load_text(const char* path, orbref_vocab** out);
int orbref_vocab_load_binary(const char* path, orbref_vocab** out);
int orbref_vocab_from_table(int n_nodes, int k, int levels, int scoring, int weighting,
                            const int32_t* parent, const uint8_t* is_leaf, const uint8_t* node_desc,
                            const double* weights, orbref_vocab** out);
void orbref_vocab_free(orbref_vocab* v);
int orbref_vocab_info(const orbref_vocab* v, int* info6);
int orbref_vocab_tables(const orbref_vocab* v, int32_t* parent, uint8_t* is_word, uint8_t* desc,
                        double* weight, uint32_t* word_id);
int orbref_vocab_transform_full(const orbref_vocab* v, const uint8_t* desc, int n, int levelsup,
                                uint32_t* bow_words, double* bow_weights, int* n_words,
                                uint32_t* node_ids, int32_t* offsets, int32_t* indices,
                                int* n_nodes);
/* Frame::isInFrustum over a MapPoint set (Frame.cc:318-374, MapPoint.cc:403-447) and
 * Tracking::SearchLocalPoints' projection + SearchByProjection (Tracking.cc:1186-1213). */
int orbref_is_in_frustum(const orbfe_frame_view* frame, const orbfe_mappoint_geometry* geom,
                         const float* tcw, float log_scale_factor, float viewing_cos_limit,
                         const orbfe_frustum_out* out, int* n_in_view);
int orbref_search_local_points(const orbfe_frame_view* frame, const orbfe_mappoint_geometry* geom,
                               const float* tcw, float log_scale_factor, float viewing_cos_limit,
                               float th, float nnratio, int32_t* best_idx, int* nmatches,
                               const orbfe_frustum_out* out, int* n_in_view);
/* One pyramid level (ORBextractor::mvImagePyramid[l]): rows x cols bytes, row stride. */
typedef struct orbref_level_view {
  const uint8_t* data;
  int rows, cols, stride;
} orbref_level_view;
/* Frame::ComputeStereoMatches (src/Frame.cc:522-700): u_right / depth per left keypoint (-1 when
 * unmatched). */
int orbref_compute_stereo_matches(const orbfe_keypoint* kl, const uint8_t* dl, int nl,
                                  const orbfe_keypoint* kr, const uint8_t* dr, int nr,
                                  const orbref_level_view* pyr_l, const orbref_level_view* pyr_r,
                                  int nlevels, const float* scale, const float* inv_scale, float mb,
                                  float mbf, float* u_right, float* depth);
/* Frame::AssignFeaturesToGrid as CSR (64 x 48 cells, cell = ix*48 + iy): cell_start[3073]. */
int orbref_build_grid(const orbfe_frame_view* frame, int32_t* cell_start, int32_t* cell_items);

/* Keyframe matchers and ComputeDistinctiveDescriptors (orbref_kf.cpp; encodings as
 * include/orbfe_keyframe.h). */
int orbref_search_by_bow_kf_frame(const orbfe_frame_view* kf, const orbfe_feature_vector* kf_fv,
                                  const orbfe_frame_view* frame, const orbfe_feature_vector* frame_fv,
                                  float nnratio, int check_ori, int32_t* match_f, int* nmatches);
int orbref_search_by_bow_kf_kf(const orbfe_frame_view* kf1, const orbfe_feature_vector* fv1,
                               const orbfe_frame_view* kf2, const orbfe_feature_vector* fv2,
                               float nnratio, int check_ori, int32_t* match12, int* nmatches);
int orbref_search_by_projection_keyframe(const orbfe_frame_view* current, const float* tcw,
                                         const orbfe_mappoint_geometry* kf_points,
                                         const float* kf_angle, float log_scale_factor, float th,
                                         int orb_dist, int check_ori, int32_t* best_idx,
                                         int* nmatches);
int orbref_search_by_projection_sim3(const orbfe_frame_view* kf, const float* scw,
                                     const orbfe_mappoint_geometry* points, float log_scale_factor,
                                     int th, int32_t* best_idx, int* nmatches);
int orbref_fuse(const orbfe_frame_view* kf, const float* tcw, const float* ow,
                const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
                int32_t* best_idx, int* n_candidates);
int orbref_fuse_sim3(const orbfe_frame_view* kf, const float* scw,
                     const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
                     int32_t* best_idx, int* nfused);
int orbref_search_by_sim3(const orbfe_frame_view* kf1, const orbfe_frame_view* kf2,
                          const orbfe_mappoint_geometry* mps1, const orbfe_mappoint_geometry* mps2,
                          const float* t1w, const float* t2w, float s12, const float* r12,
                          const float* t12, float lsf1, float lsf2, float th, int32_t* match12,
                          int* nfound);
int orbref_search_for_initialization(const orbfe_frame_view* f1, const orbfe_frame_view* f2,
                                     float* prev_matched, int window, float nnratio, int check_ori,
                                     int32_t* match12, int* nmatches);
long long orbref_check_predict_scale(float lsf, int nlevels, const float* thr, uint32_t lo_bits,
                                     uint32_t hi_bits, long long* non_monotone);
int orbref_compute_distinctive_descriptors(int n_points, const int32_t* offsets,
                                           const uint8_t* descriptors, int32_t* best_index);

#ifdef __cplusplus
}
#endif
#endif
