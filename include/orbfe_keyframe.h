/*
 * orbfe_keyframe.h -- the remaining ORBmatcher searches (keyframe / relocalisation / loop-closing
 * matchers) and MapPoint::ComputeDistinctiveDescriptors on MI355X (liborbfe.so, gfx950).
 *
 * Replaces, in the reference (lreithmayr/ORB_SLAM2_2021, src/ORBmatcher.cc unless noted):
 *   SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)                          :165-293
 *   SearchByProjection(KeyFrame*, cv::Mat Scw, vector<MapPoint*>, vector<MapPoint*>&, int th)
 *                                                                               :295-412
 *   SearchForInitialization(Frame&, Frame&, vector<cv::Point2f>&, vector<int>&, int)
 *                                                                               :414-534
 *   SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)                       :536-669
 *   Fuse(KeyFrame*, const vector<MapPoint*>&, float th)                         :841-991
 *   Fuse(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, float, vector<MapPoint*>&)
 *                                                                               :993-1120
 *   SearchBySim3(KeyFrame*, KeyFrame*, vector<MapPoint*>&, float s12, R12, t12, float th)
 *                                                                               :1122-1346
 *   SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, float th, int ORBdist)
 *                                                                               :1493-1625
 *   MapPoint::ComputeDistinctiveDescriptors()                     src/MapPoint.cc:272-337
 *   MapPoint::PredictScale(float, KeyFrame* / Frame*)             src/MapPoint.cc:415-447
 *
 * Conventions shared with orbfe.h:
 *   - A KeyFrame is an orbfe_frame_view. Its min_x..max_y are the KeyFrame's own `const int`
 *     mnMinX.. (KeyFrame.h:202-205) as floats; they bound IsInImage (KeyFrame.cc:627-630) and
 *     GetFeaturesInArea (KeyFrame.cc:586-625). Its mGrid is the Frame's, built with the Frame's
 *     float bounds: set grid_origin_set = 1 and grid_min_x/y = those bounds (they differ only for
 *     a distorted camera).
 *   - mp_state per keypoint is what the matcher reads of the keypoint's MapPoint:
 *     ORBFE_MP_NONE = NULL; ORBFE_MP_BAD = non-NULL with isBad(); otherwise PRESENT / OBSERVED.
 *   - MapPoint inputs use orbfe_mappoint_geometry (orbfe_frustum.h) with the flags below.
 *   - log_scale_factor = the KeyFrame's / Frame's mfLogScaleFactor (= logf(scale factor)).
 *   - The matchers never mutate the map: they return what the reference would have assigned, and
 *     the adapter applies it. Where the reference's loop reads state that the
 *     adapter's own application changes (Fuse), the return value says so.
 * All buffers are host memory; calls block until the results are back.
 */
#ifndef ORBFE_KEYFRAME_H
#define ORBFE_KEYFRAME_H
#include <stdint.h>

#include "orbfe.h"
#include "orbfe_frustum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mp_state value: the keypoint holds a MapPoint whose isBad() is true. */
#define ORBFE_MP_BAD 3

/* orbfe_mappoint_geometry.flags bit: the MapPoint is skipped by the loop's own test --
 * in sAlreadyFound / spAlreadyFound (SearchByProjection :1519, :326; Fuse(Scw) :1025),
 * pMP->IsInKeyFrame(pKF) (Fuse :865) or vbAlreadyMatched1/2 (SearchBySim3 :1172, :1252). */
#define ORBFE_MPF_SKIP 64u

/* SearchByBoW(pKF, F, vpMapPointMatches) (:165-293). match_f[F.N]: the KF keypoint whose
 * MapPoint the reference puts in vpMapPointMatches[k] (-1 = NULL), after the rotation filter.
 * kf.mp_state: the KF's GetMapPointMatches() (NONE / BAD / present). F's mp_state is not read. */
int orbfe_search_by_bow_kf_frame(orbfe_matcher* m, const orbfe_frame_view* kf,
                                 const orbfe_feature_vector* kf_fv, const orbfe_frame_view* frame,
                                 const orbfe_feature_vector* frame_fv, int32_t* match_f,
                                 int* nmatches);

/* Tracking::Relocalization's loop (Tracking.cc) of SearchByBoW(vpCandidateKFs[i], F, ...) over
 * n_kf keyframes against one frame, in one launch: match_f[i * F.N + k], nmatches[i]. */
int orbfe_search_by_bow_kf_frame_multi(orbfe_matcher* m, int n_kf, const orbfe_frame_view* kfs,
                                       const orbfe_feature_vector* kf_fvs,
                                       const orbfe_frame_view* frame,
                                       const orbfe_feature_vector* frame_fv, int32_t* match_f,
                                       int32_t* nmatches);

/* SearchByBoW(pKF1, pKF2, vpMatches12) (:536-669). match12[KF1.N]: idx2 whose MapPoint the
 * reference puts in vpMatches12[idx1], or -1. Both mp_state arrays are read (NONE / BAD). */
int orbfe_search_by_bow_kf_kf(orbfe_matcher* m, const orbfe_frame_view* kf1,
                              const orbfe_feature_vector* fv1, const orbfe_frame_view* kf2,
                              const orbfe_feature_vector* fv2, int32_t* match12, int* nmatches);

/* SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1493-1625).
 * kf_points: pKF->GetMapPointMatches() by KF keypoint (flags PRESENT, BAD, SKIP = in
 * sAlreadyFound; world_pos, min/max_distance, descriptors; normal unused); kf_angle: the KF's
 * mvKeysUn[i].angle. current.mp_state: CurrentFrame.mvpMapPoints (any non-NULL blocks).
 * tcw_cur: CurrentFrame.mTcw rows 0..2. best_idx as orbfe_search_by_projection_lastframe
 * (k >= 0 assigned, <= -2 assigned then undone by the rotation filter). */
int orbfe_search_by_projection_keyframe(orbfe_matcher* m, const orbfe_frame_view* current,
                                        const float* tcw_cur,
                                        const orbfe_mappoint_geometry* kf_points,
                                        const float* kf_angle, float log_scale_factor, float th,
                                        int orb_dist, int32_t* best_idx, int* nmatches);

/* SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (:295-412). scw: rows 0..2 of the 4x4
 * Sim3 (3x4 row-major). kf.mp_state: vpMatched (non-NULL = taken). points: flags BAD, SKIP (in
 * spAlreadyFound). best_idx[i]: KF keypoint the reference sets vpMatched[k] = vpPoints[i] on, or
 * -1; apply in ascending i. */
int orbfe_search_by_projection_sim3(orbfe_matcher* m, const orbfe_frame_view* kf, const float* scw,
                                    const orbfe_mappoint_geometry* points, float log_scale_factor,
                                    int th, int32_t* best_idx, int* nmatches);

/* Fuse(pKF, vpMapPoints, th) (:841-991). tcw: pKF->GetPose() rows 0..2; ow: GetCameraCenter().
 * points: flags PRESENT (non-NULL), BAD, SKIP (IsInKeyFrame(pKF)). best_idx[i]: the keypoint
 * the reference fuses vpMapPoints[i] into (bestDist <= TH_LOW), or -1. The search reads no map
 * state the loop changes; the adapter applies in ascending i and re-tests isBad() /
 * IsInKeyFrame() at that time (an earlier Replace can change them), counting nFused itself.
 * *n_candidates = entries with best_idx >= 0. */
int orbfe_fuse(orbfe_matcher* m, const orbfe_frame_view* kf, const float* tcw, const float* ow,
               const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
               int32_t* best_idx, int* n_candidates);

/* Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:993-1120). points: flags BAD, SKIP (in
 * pKF->GetMapPoints()). best_idx[i]: keypoint matched by vpPoints[i] or -1; the adapter applies
 * in ascending i (replace when pKF->GetMapPoint(k) is set and not bad, else add). *nfused = the
 * reference's return value. */
int orbfe_fuse_sim3(orbfe_matcher* m, const orbfe_frame_view* kf, const float* scw,
                    const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
                    int32_t* best_idx, int* nfused);

/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (:1122-1346). mps1 / mps2: the two
 * KeyFrames' GetMapPointMatches() by keypoint (flags PRESENT, BAD, SKIP = vbAlreadyMatched).
 * t1w, t2w: the KeyFrames' poses rows 0..2; r12 row-major 3x3; t12[3]. Both projections use
 * KF1's fx, fy, cx, cy, as the reference does. match12[KF1.N]: idx2 where the two searches
 * agree (vpMatches12[i1] = vpMapPoints2[idx2]), else -1. *nfound = the return value. */
int orbfe_search_by_sim3(orbfe_matcher* m, const orbfe_frame_view* kf1, const orbfe_frame_view* kf2,
                         const orbfe_mappoint_geometry* mps1, const orbfe_mappoint_geometry* mps2,
                         const float* t1w, const float* t2w, float s12, const float* r12,
                         const float* t12, float log_scale_factor1, float log_scale_factor2,
                         float th, int32_t* match12, int* nfound);

/* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (:414-534).
 * prev_matched: N1 x 2 floats, updated in place as the reference does (:528-531);
 * match12[N1] = vnMatches12. */
int orbfe_search_for_initialization(orbfe_matcher* m, const orbfe_frame_view* f1,
                                    const orbfe_frame_view* f2, float* prev_matched,
                                    int window_size, int32_t* match12, int* nmatches);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:272-337) for n_points MapPoints:
 * point i's descriptors (its good KeyFrames' rows, in mObservations order) are
 * descriptors[offsets[i] .. offsets[i+1]) (32 B each); best_index[i] = BestIdx within them
 * (-1 for a point with none, where the reference returns early). */
int orbfe_compute_distinctive_descriptors(orbfe_matcher* m, int n_points, const int32_t* offsets,
                                          const uint8_t* descriptors, int32_t* best_index);

/* Device-resident form of the above (all pointers device memory, async on `stream`, NULL = the
 * matcher's stream). */
int orbfe_compute_distinctive_descriptors_device(orbfe_matcher* m, int n_points,
                                                 const int32_t* d_offsets,
                                                 const uint8_t* d_descriptors,
                                                 int32_t* d_best_index, void* stream);

/* MapPoint::PredictScale as a table: with mfLogScaleFactor = log_scale_factor and nlevels
 * levels, nScale(ratio) = #{k : ratio >= thresholds[k-1], 1 <= k < nlevels} for ratio =
 * mfMaxDistance / dist > 0. thresholds[k-1] is the smallest float ratio with
 * ceil(logf(ratio) / log_scale_factor) >= k, found with the host's logf: the device kernels
 * compare against these instead of evaluating log. */
int orbfe_predict_scale_thresholds(float log_scale_factor, int nlevels, float* thresholds);

#ifdef __cplusplus
}
#endif
#endif
