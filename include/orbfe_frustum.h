/*
 * orbfe_frustum.h -- Frame::isInFrustum over the local map, and Tracking::SearchLocalPoints'
 * projection + SearchByProjection as one device pass (liborbfe.so, gfx950).
 *
 * Replaces, in the reference (lreithmayr/ORB_SLAM2_2021):
 *   Frame::isInFrustum(MapPoint*, float viewingCosLimit)   src/Frame.cc:318-374
 *   MapPoint::PredictScale(float, Frame*)                  src/MapPoint.cc:432-447
 *   MapPoint::Get{Min,Max}DistanceInvariance               src/MapPoint.cc:403-413
 *   the projection loop + SearchByProjection of Tracking::SearchLocalPoints
 *                                                          src/Tracking.cc:1186-1213
 * Float algebra follows the reference's cv::Mat CV_32F operations: the
 * 3x3 gemm Rcw*P + tcw and -Rcw^T*tcw accumulate in double and round once, cv::norm and
 * Mat::dot accumulate squares / products in double.
 */
#ifndef ORBFE_FRUSTUM_H
#define ORBFE_FRUSTUM_H
#include <stdint.h>

#include "orbfe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* MapPoint::mnLastFrameSeen == CurrentFrame.mnId: already matched in this frame, so
 * SearchLocalPoints skips its projection (Tracking.cc:1193-1194) and mbTrackInView stays false. */
#define ORBFE_MPF_SEEN 32u

/* The local map's MapPoints as isInFrustum reads them. */
typedef struct orbfe_mappoint_geometry {
  int32_t m;
  const uint8_t* flags;         /* ORBFE_MPF_BAD | ORBFE_MPF_SEEN (others ignored) */
  const float* world_pos;       /* GetWorldPos(), m x 3 */
  const float* normal;          /* GetNormal(), m x 3 */
  const float* min_distance;    /* mfMinDistance (isInFrustum uses 0.8f * it) */
  const float* max_distance;    /* mfMaxDistance (1.2f * it; PredictScale uses it as is) */
  const uint8_t* descriptors;   /* GetDescriptor(), m x 32 (SearchByProjection only) */
} orbfe_mappoint_geometry;

/* Per-MapPoint outputs: the members isInFrustum writes (Frame.cc:365-371). */
typedef struct orbfe_frustum_out {
  uint8_t* flags;      /* input flags with ORBFE_MPF_TRACK_IN_VIEW = mbTrackInView */
  float* proj_x;       /* mTrackProjX   (written when in view) */
  float* proj_y;       /* mTrackProjY */
  float* proj_xr;      /* mTrackProjXR */
  int32_t* level;      /* mnTrackScaleLevel */
  float* view_cos;     /* mTrackViewCos */
} orbfe_frustum_out;

/* isInFrustum(pMP, viewing_cos_limit) for every MapPoint of geom not flagged BAD or SEEN, with
 * the frame's camera (F: fx, fy, cx, cy, bf, min/max x/y, nlevels), pose tcw (CurrentFrame.mTcw
 * rows 0..2, 3x4 row-major) and mfLogScaleFactor. *n_in_view = how many passed (nToMatch,
 * Tracking.cc:1197-1201). Blocking. The geometry arrays (and the frame view's arrays) may be host
 * memory or device memory: device inputs -- a local map kept resident in HBM -- are copied on the
 * device instead of being staged through pinned host memory. Outputs are host buffers. */
int orbfe_is_in_frustum(orbfe_matcher* m, const orbfe_frame_view* frame,
                        const orbfe_mappoint_geometry* geom, const float* tcw,
                        float log_scale_factor, float viewing_cos_limit,
                        const orbfe_frustum_out* out, int* n_in_view);

/* Tracking::SearchLocalPoints' hot part: isInFrustum(pMP, 0.5) over the local map, then, when
 * any MapPoint is in view, SearchByProjection(CurrentFrame, vpLocalMapPoints, th) on the device
 * without a host round trip. best_idx as orbfe_search_by_projection_local (all -1 when nothing is
 * in view, as the reference skips the matcher). out may be NULL or have NULL members. */
int orbfe_search_local_points(orbfe_matcher* m, const orbfe_frame_view* frame,
                              const orbfe_mappoint_geometry* geom, const float* tcw,
                              float log_scale_factor, float viewing_cos_limit, float th,
                              int32_t* best_idx, int* nmatches, const orbfe_frustum_out* out,
                              int* n_in_view);

#ifdef __cplusplus
}
#endif
#endif
