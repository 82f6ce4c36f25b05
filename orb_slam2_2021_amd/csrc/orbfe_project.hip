// orbfe_project.hip -- the projection searches of ORBmatcher outside the tracking hot loop, on the
// SearchByProjection engine of orbfe_match.hip (gfx950, wave64).
//
// Reference: src/ORBmatcher.cc of lreithmayr/ORB_SLAM2_2021.
//   SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)  :1493-1625  (relocalisation)
//   SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) :295-412  (loop closing)
//   Fuse(KeyFrame*, vpMapPoints, th)                           :841-991  (local mapping)
//   Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)         :993-1120 (loop closing)
//   SearchBySim3(KF1, KF2, vpMatches12, s12, R12, t12, th)     :1122-1346
// Every one is "project MapPoint i, then take the first-minimum Hamming distance over the
// window's keypoints at the predicted levels". k_proj_queries turns each MapPoint into an
// SbpQuery (thread per MapPoint: the pose algebra, the visibility tests and PredictScale); the
// engine then does the window walk + distances (16 lanes per query) and, where an assignment
// blocks later MapPoints (vpMatched, mvpMapPoints), the claim-order fixpoint.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/orbfe.h"
#include "../../include/orbfe_frustum.h"
#include "../../include/orbfe_keyframe.h"
#include "orbfe_device.h"
#include "orbfe_match_internal.h"
#include "orbfe_ktimer.h"

using namespace orbfe_mi;

namespace {
enum ProjKind { PQ_RELOC = 0, PQ_SBP_SIM3 = 1, PQ_FUSE = 2, PQ_FUSE_SIM3 = 3, PQ_SIM3_DIR = 4 };

struct ProjQueryArgs {
  int m, kind;
  const uint8_t* flags;
  const float* pos;
  const float* normal;
  const float* min_d;
  const float* max_d;
  float R[9], t[3], Ow[3];  // world -> camera (SIM3_DIR: world -> camera A)
  float R2[9], t2[3];       // SIM3_DIR: camera A -> camera B (sR21 / t21 or sR12 / t12)
  float fx, fy, cx, cy, bf;
  float min_x, max_x, min_y, max_y;  // target image bounds
  int nlevels;
  const float* scale_factors;        // target's mvScaleFactors (device)
  float th;
  float scale_thr[ORBFE_MAX_LEVELS_M];
  SbpQuery* q;
};

__device__ __forceinline__ float norm3_d(float x, float y, float z) {  // cv::norm, double accumulation
  double s = (double)x * (double)x;
  s += (double)y * (double)y;
  s += (double)z * (double)z;
  return (float)sqrt(s);
}
__device__ __forceinline__ double dot3_d(float x, float y, float z, const float* n) {  // Mat::dot
  double s = (double)x * (double)n[0];
  s += (double)y * (double)n[1];
  s += (double)z * (double)n[2];
  return s;
}

__global__ __launch_bounds__(256) void k_proj_queries(ProjQueryArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.m) return;
  SbpQuery q = {};
  q.gate = SBP_GATE_NONE;
  const uint8_t fl = a.flags[i];
  const int kind = a.kind;
  bool ok = !(fl & (ORBFE_MPF_BAD | ORBFE_MPF_SKIP));
  if (kind != PQ_SBP_SIM3 && kind != PQ_FUSE_SIM3) ok = ok && (fl & ORBFE_MPF_PRESENT);
  if (ok) {
    const float X = a.pos[3 * i], Y = a.pos[3 * i + 1], Z = a.pos[3 * i + 2];
    float xc = gemv3_d(a.R, X, Y, Z, a.t[0]);
    float yc = gemv3_d(a.R + 3, X, Y, Z, a.t[1]);
    float zc = gemv3_d(a.R + 6, X, Y, Z, a.t[2]);
    if (kind == PQ_SIM3_DIR) {  // p3Dc2 = sR21 * p3Dc1 + t21 (:1179-1180) and the mirror (:1259-1260)
      const float x2 = gemv3_d(a.R2, xc, yc, zc, a.t2[0]);
      const float y2 = gemv3_d(a.R2 + 3, xc, yc, zc, a.t2[1]);
      const float z2 = gemv3_d(a.R2 + 6, xc, yc, zc, a.t2[2]);
      xc = x2;
      yc = y2;
      zc = z2;
    }
    float u, v, ur = 0.f;
    if (kind == PQ_RELOC) {  // :1525-1535: no depth test; Frame bounds, inclusive
      const float invzc = (float)(1.0 / (double)zc);
      u = a.fx * xc * invzc + a.cx;
      v = a.fy * yc * invzc + a.cy;
      ok = !(u < a.min_x || u > a.max_x) && !(v < a.min_y || v > a.max_y);
    } else {  // depth must be positive, then KeyFrame::IsInImage (KeyFrame.cc:627-630)
      ok = !(zc < 0.0f);
      // 1 / z in float (:340, :875) or 1.0 / z in double (:1039, :1186, :1266)
      const float invz = (kind == PQ_SBP_SIM3 || kind == PQ_FUSE) ? 1.0f / zc : (float)(1.0 / (double)zc);
      const float x = xc * invz, y = yc * invz;
      u = a.fx * x + a.cx;
      v = a.fy * y + a.cy;
      ok = ok && u >= a.min_x && u < a.max_x && v >= a.min_y && v < a.max_y;
      ur = u - a.bf * invz;  // Fuse (:886)
    }
    if (ok) {
      const float maxDistance = 1.2f * a.max_d[i];  // Get{Max,Min}DistanceInvariance
      const float minDistance = 0.8f * a.min_d[i];
      float POx, POy, POz;
      if (kind == PQ_SIM3_DIR) {  // dist3D = cv::norm(p3Dc2) (:1199)
        POx = xc;
        POy = yc;
        POz = zc;
      } else {
        POx = X - a.Ow[0];
        POy = Y - a.Ow[1];
        POz = Z - a.Ow[2];
      }
      const float dist = norm3_d(POx, POy, POz);
      ok = !(dist < minDistance || dist > maxDistance);
      if (ok && kind != PQ_RELOC && kind != PQ_SIM3_DIR)  // viewing angle < 60 deg (:363, :900, :1062)
        ok = !(dot3_d(POx, POy, POz, a.normal + 3 * i) < 0.5 * (double)dist);
      if (ok) {
        const int pred = predict_scale_dev(a.max_d[i], dist, a.scale_thr, a.nlevels);
        const float radius = a.th * a.scale_factors[pred];
        q.x = u;
        q.y = v;
        q.r = radius;
        q.xr = ur;
        q.er_lim = 0.f;
        q.min_level = pred - 1;  // kpLevel < pred - 1 || kpLevel > pred (:389, :927, :1087, :1227)
        q.max_level = kind == PQ_RELOC ? pred + 1 : pred;  // GetFeaturesInArea(.., pred-1, pred+1) (:1553)
        q.gate = kind == PQ_FUSE ? SBP_GATE_FUSE : SBP_GATE_NONE;
        // an assignment takes the keypoint for later MapPoints: CurrentFrame.mvpMapPoints (:1583),
        // vpMatched (:405); Fuse and SearchBySim3 never skip a matched keypoint
        q.flags = 1 | ((kind == PQ_RELOC || kind == PQ_SBP_SIM3) ? 2 : 0);
      }
    }
  }
  a.q[i] = q;
}

// SearchBySim3's agreement check (:1328-1343)
__global__ __launch_bounds__(256) void k_sim3_agree(const int32_t* m1, const int32_t* m2, int n1, int n2,
                                                     int32_t* match12, int32_t* nfound) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool ok = false;
  if (i < n1) {
    const int idx2 = m1[i];
    ok = idx2 >= 0 && idx2 < n2 && m2[idx2] == i;
    match12[i] = ok ? idx2 : -1;
  }
  __shared__ int s_c[4];
  const int c = __popcll(wave_ballot(ok));
  if (lane_id() == 0) s_c[wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0 && s_c[0] + s_c[1] + s_c[2] + s_c[3]) atomicAdd(nfound, s_c[0] + s_c[1] + s_c[2] + s_c[3]);
}

// ---- host -----------------------------------------------------------------------------------------
struct Pose {
  float R[9], t[3], Ow[3];
};
Pose pose_from(const float* T) {  // [R|t] rows; Ow = -R^T t (gemm alpha = -1, double accumulation)
  Pose p;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) p.R[3 * r + c] = T[4 * r + c];
    p.t[r] = T[4 * r + 3];
  }
  for (int i = 0; i < 3; i++) {
    double s = (double)p.R[i] * (double)p.t[0];
    s += (double)p.R[3 + i] * (double)p.t[1];
    s += (double)p.R[6 + i] * (double)p.t[2];
    p.Ow[i] = -(float)s;
  }
  return p;
}
// Scw decomposition (:308-312, :1006-1010): scw = sqrt(row0 . row0) (Mat::dot in double); sRcw / scw
// and col(3) / scw are MatExpr scalings, evaluated by convertTo with the float factor 1 / scw.
Pose pose_from_sim3(const float* S) {
  double d = 0.0;
  for (int k = 0; k < 3; k++) d += (double)S[k] * (double)S[k];
  const float scw = (float)std::sqrt(d);
  const float f = (float)(1.0 / (double)scw);
  float T[12];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 4; c++) T[4 * r + c] = S[4 * r + c] * f;
  return pose_from(T);
}

bool geometry_ok(const orbfe_mappoint_geometry* g, bool need_normal) {
  return g && g->m >= 0 &&
         (g->m == 0 || (g->flags && g->world_pos && g->min_distance && g->max_distance && g->descriptors &&
                        (!need_normal || g->normal)));
}

struct GeomOffsets {
  size_t flags, pos, normal, mind, maxd;
};
GeomOffsets plan_geom(Arena& ar, const orbfe_mappoint_geometry* g, bool need_normal) {
  const size_t m1 = (size_t)std::max(g->m, 1);
  GeomOffsets o;
  o.flags = ar.add(m1);
  o.pos = ar.add(12 * m1);
  o.normal = ar.add(need_normal ? 12 * m1 : 0);
  o.mind = ar.add(4 * m1);
  o.maxd = ar.add(4 * m1);
  return o;
}
void stage_geom(orbfe_matcher* m, const GeomOffsets& o, const orbfe_mappoint_geometry* g, bool need_normal,
                ProjQueryArgs& qa) {
  uint8_t* A = m->arena;
  const size_t n = (size_t)g->m;
  if (n) {
    stage_h2d(m, A + o.flags, g->flags, n);
    stage_h2d(m, A + o.pos, g->world_pos, 12 * n);
    if (need_normal) stage_h2d(m, A + o.normal, g->normal, 12 * n);
    stage_h2d(m, A + o.mind, g->min_distance, 4 * n);
    stage_h2d(m, A + o.maxd, g->max_distance, 4 * n);
  }
  qa.m = g->m;
  qa.flags = A + o.flags;
  qa.pos = (const float*)(A + o.pos);
  qa.normal = need_normal ? (const float*)(A + o.normal) : nullptr;
  qa.min_d = (const float*)(A + o.mind);
  qa.max_d = (const float*)(A + o.maxd);
}
void set_camera(ProjQueryArgs& qa, const orbfe_frame_view* cam, const orbfe_frame_view* target,
                const orbfe_frame_view& d_target, float lsf, float th) {
  qa.fx = cam->fx;
  qa.fy = cam->fy;
  qa.cx = cam->cx;
  qa.cy = cam->cy;
  qa.bf = cam->bf;
  qa.min_x = target->min_x;
  qa.max_x = target->max_x;
  qa.min_y = target->min_y;
  qa.max_y = target->max_y;
  qa.nlevels = target->nlevels;
  qa.scale_factors = d_target.scale_factors;
  qa.th = th;
  predict_scale_table(lsf, target->nlevels, qa.scale_thr);
}
void set_pose(ProjQueryArgs& qa, const Pose& p) {
  std::memcpy(qa.R, p.R, sizeof(p.R));
  std::memcpy(qa.t, p.t, sizeof(p.t));
  std::memcpy(qa.Ow, p.Ow, sizeof(p.Ow));
}
void launch_queries(orbfe_matcher* m, const SbpPlan& p, ProjQueryArgs qa) {
  qa.q = (SbpQuery*)(m->arena + p.oq);
  if (qa.m > 0) ORBFE_LAUNCH("k_proj_queries", k_proj_queries, dim3((qa.m + 255) / 256), dim3(256), 0, m->stream, qa);
}

// One projection search: plan, stage frame + points, queries, engine, fetch.
int run_projection(orbfe_matcher* m, const orbfe_frame_view* target, const orbfe_mappoint_geometry* pts,
                   bool need_normal, const float* h_qangle, ProjQueryArgs qa, const SbpMode& md,
                   const orbfe_frame_view* cam, float lsf, float th, int32_t* best_idx, int* count) {
  hipSetDevice(m->device);
  Arena ar;
  SbpPlan p;
  sbp_plan_inputs(ar, target, pts->m, sbp_cand_cap(m), p);
  const GeomOffsets go = plan_geom(ar, pts, need_normal);
  sbp_plan_scratch(ar, target, p);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  orbfe_frame_view dT;
  if ((st = sbp_stage(m, p, target, pts->m ? pts->descriptors : nullptr, h_qangle, &dT))) return st;
  stage_geom(m, go, pts, need_normal, qa);
  if ((st = flush_h2d(m))) return st;
  set_camera(qa, cam, target, dT, lsf, th);
  launch_queries(m, p, qa);
  if ((st = sbp_launch(m, p, target, dT, md, true))) return st;
  return sbp_fetch(m, p, best_idx, count, target, &dT, &md);
}

bool target_ok(const orbfe_frame_view* f) { return frame_ok(f) && levels_ok(f->keys_un, f->n, f->nlevels); }
}  // namespace

extern "C" int orbfe_search_by_projection_keyframe(orbfe_matcher* m, const orbfe_frame_view* current,
                                                   const float* tcw_cur, const orbfe_mappoint_geometry* kf_points,
                                                   const float* kf_angle, float log_scale_factor, float th,
                                                   int orb_dist, int32_t* best_idx, int* nmatches) {
  if (!m || !target_ok(current) || !tcw_cur || !geometry_ok(kf_points, false) || !nmatches ||
      (kf_points->m > 0 && (!best_idx || !kf_angle)))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_projection_keyframe: bad argument");
  ProjQueryArgs qa;
  std::memset(&qa, 0, sizeof(qa));
  qa.kind = PQ_RELOC;
  set_pose(qa, pose_from(tcw_cur));
  // first minimum with bestDist <= ORBdist; any non-NULL mvpMapPoints entry blocks (:1567)
  const SbpMode md{1, orb_dist, SBP_BLOCK_ANY, m->check_ori};
  return run_projection(m, current, kf_points, false, kf_angle, qa, md, current, log_scale_factor, th, best_idx,
                        nmatches);
}

extern "C" int orbfe_search_by_projection_sim3(orbfe_matcher* m, const orbfe_frame_view* kf, const float* scw,
                                               const orbfe_mappoint_geometry* points, float log_scale_factor,
                                               int th, int32_t* best_idx, int* nmatches) {
  if (!m || !target_ok(kf) || !scw || !geometry_ok(points, true) || !nmatches || (points->m > 0 && !best_idx))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_projection_sim3: bad argument");
  ProjQueryArgs qa;
  std::memset(&qa, 0, sizeof(qa));
  qa.kind = PQ_SBP_SIM3;
  set_pose(qa, pose_from_sim3(scw));
  const SbpMode md{1, TH_LOW, SBP_BLOCK_ANY, 0};  // vpMatched: any non-NULL entry blocks (:384)
  return run_projection(m, kf, points, true, nullptr, qa, md, kf, log_scale_factor, (float)th, best_idx,
                        nmatches);
}

extern "C" int orbfe_fuse(orbfe_matcher* m, const orbfe_frame_view* kf, const float* tcw, const float* ow,
                          const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
                          int32_t* best_idx, int* n_candidates) {
  if (!m || !target_ok(kf) || !kf->level_sigma2 || !tcw || !ow || !geometry_ok(points, true) || !n_candidates ||
      (points->m > 0 && !best_idx))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_fuse: bad argument");
  ProjQueryArgs qa;
  std::memset(&qa, 0, sizeof(qa));
  qa.kind = PQ_FUSE;
  Pose p = pose_from(tcw);
  std::memcpy(p.Ow, ow, sizeof(p.Ow));  // pKF->GetCameraCenter() (:852)
  set_pose(qa, p);
  const SbpMode md{1, TH_LOW, SBP_BLOCK_NONE, 0, 1};  // no claims: nothing blocks
  return run_projection(m, kf, points, true, nullptr, qa, md, kf, log_scale_factor, th, best_idx, n_candidates);
}

extern "C" int orbfe_fuse_sim3(orbfe_matcher* m, const orbfe_frame_view* kf, const float* scw,
                               const orbfe_mappoint_geometry* points, float log_scale_factor, float th,
                               int32_t* best_idx, int* nfused) {
  if (!m || !target_ok(kf) || !scw || !geometry_ok(points, true) || !nfused || (points->m > 0 && !best_idx))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_fuse_sim3: bad argument");
  ProjQueryArgs qa;
  std::memset(&qa, 0, sizeof(qa));
  qa.kind = PQ_FUSE_SIM3;
  set_pose(qa, pose_from_sim3(scw));
  const SbpMode md{1, TH_LOW, SBP_BLOCK_NONE, 0, 1};
  return run_projection(m, kf, points, true, nullptr, qa, md, kf, log_scale_factor, th, best_idx, nfused);
}

extern "C" int orbfe_search_by_sim3(orbfe_matcher* m, const orbfe_frame_view* kf1, const orbfe_frame_view* kf2,
                                    const orbfe_mappoint_geometry* mps1, const orbfe_mappoint_geometry* mps2,
                                    const float* t1w, const float* t2w, float s12, const float* r12,
                                    const float* t12, float lsf1, float lsf2, float th, int32_t* match12,
                                    int* nfound) {
  if (!m || !target_ok(kf1) || !target_ok(kf2) || !geometry_ok(mps1, false) || !geometry_ok(mps2, false) ||
      !t1w || !t2w || !r12 || !t12 || !nfound || mps1->m != kf1->n || mps2->m != kf2->n ||
      (kf1->n > 0 && !match12))
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_search_by_sim3: bad argument");
  hipSetDevice(m->device);
  // sR12 = s12 * R12; sR21 = (1 / s12) * R12^T; t21 = -sR21 * t12 (:1139-1141)
  float sR12[9], sR21[9], t21[3];
  const float inv_s = (float)(1.0 / (double)s12);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      sR12[3 * r + c] = r12[3 * r + c] * s12;
      sR21[3 * r + c] = r12[3 * c + r] * inv_s;
    }
  for (int r = 0; r < 3; r++) {
    double s = (double)sR21[3 * r] * (double)t12[0];
    s += (double)sR21[3 * r + 1] * (double)t12[1];
    s += (double)sR21[3 * r + 2] * (double)t12[2];
    t21[r] = -(float)s;
  }
  // two searches (KF1's points into KF2, KF2's into KF1) in one arena, then the agreement kernel
  Arena ar;
  SbpPlan p1, p2;
  sbp_plan_inputs(ar, kf2, mps1->m, sbp_cand_cap(m), p1);
  sbp_plan_inputs(ar, kf1, mps2->m, sbp_cand_cap(m), p2);
  const GeomOffsets g1 = plan_geom(ar, mps1, false), g2 = plan_geom(ar, mps2, false);
  sbp_plan_scratch(ar, kf2, p1);
  sbp_plan_scratch(ar, kf1, p2);
  const size_t om = ar.add(4 * (size_t)std::max(kf1->n, 1)), on = ar.add(4);
  int st = ensure_arena(m, ar.total);
  if (st) return st;
  uint8_t* A = m->arena;
  orbfe_frame_view d2, d1;
  if ((st = sbp_stage(m, p1, kf2, mps1->m ? mps1->descriptors : nullptr, nullptr, &d2))) return st;
  if ((st = sbp_stage(m, p2, kf1, mps2->m ? mps2->descriptors : nullptr, nullptr, &d1))) return st;
  ProjQueryArgs q1, q2;
  std::memset(&q1, 0, sizeof(q1));
  std::memset(&q2, 0, sizeof(q2));
  stage_geom(m, g1, mps1, false, q1);
  stage_geom(m, g2, mps2, false, q2);
  if ((st = flush_h2d(m))) return st;
  ORBFE_HIP_CHECK(hipMemsetAsync(A + on, 0, 4, m->stream));
  q1.kind = q2.kind = PQ_SIM3_DIR;
  const Pose P1 = pose_from(t1w), P2 = pose_from(t2w);
  set_pose(q1, P1);
  std::memcpy(q1.R2, sR21, sizeof(sR21));
  std::memcpy(q1.t2, t21, sizeof(t21));
  set_pose(q2, P2);
  std::memcpy(q2.R2, sR12, sizeof(sR12));
  std::memcpy(q2.t2, t12, sizeof(float) * 3);
  set_camera(q1, kf1, kf2, d2, lsf2, th);  // both directions project with KF1's fx, fy, cx, cy
  set_camera(q2, kf1, kf1, d1, lsf1, th);
  launch_queries(m, p1, q1);
  launch_queries(m, p2, q2);
  const SbpMode md{1, TH_HIGH, SBP_BLOCK_NONE, 0, 1};
  if ((st = sbp_launch(m, p1, kf2, d2, md))) return st;
  if ((st = sbp_launch(m, p2, kf1, d1, md))) return st;
  if (kf1->n > 0)
    ORBFE_LAUNCH("k_sim3_agree", k_sim3_agree, dim3((kf1->n + 255) / 256), dim3(256), 0, m->stream,
                       (const int32_t*)(A + p1.obest), (const int32_t*)(A + p2.obest), kf1->n, kf2->n,
                       (int32_t*)(A + om), (int32_t*)(A + on));
  ORBFE_HIP_CHECK(hipGetLastError());
  int32_t nf = 0;
  if (kf1->n > 0) orbfe_mi::stage_d2h(m, match12, A + om, 4 * (size_t)kf1->n);
  orbfe_mi::stage_d2h(m, &nf, A + on, 4);
  if ((st = orbfe_mi::fetch_d2h(m))) return st;
  *nfound = nf;
  return ORBFE_OK;
}
