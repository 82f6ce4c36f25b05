// orbref_kf.cpp -- CPU restatement of the remaining ORBmatcher searches and
// MapPoint::ComputeDistinctiveDescriptors (TEST INFRASTRUCTURE ONLY: loaded by tests/ and
// bench.py's cpu_baseline leg as the checker, never by the product path).
//
// Each function follows the reference loop statement by statement (lreithmayr/ORB_SLAM2_2021,
// src/ORBmatcher.cc unless noted) and returns what the reference writes, in the encodings of
// include/orbfe_keyframe.h. Float algebra: scalar float with no contraction; cv::Mat CV_32F
// gemm / norm / dot accumulate in double -- recalled OpenCV behaviour,
// parity unpinned at that boundary like the rest of the oracle.
#include <climits>

#include "../include/orbfe_keyframe.h"
#include "orbref.h"
#include "orbref_match.h"

using namespace orbref_m;

namespace {
struct Pose {
  float R[9], t[3], Ow[3];
};

// [R|t] rows 0..2 (3x4 row-major) and Ow = -R^T t (gemm with alpha = -1, double accumulation)
Pose pose_from(const float* T) {
  Pose p;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) p.R[3 * r + c] = T[4 * r + c];
    p.t[r] = T[4 * r + 3];
  }
  for (int i = 0; i < 3; i++) {
    const float col[3] = {p.R[i], p.R[3 + i], p.R[6 + i]};
    p.Ow[i] = -gemv_row(col, p.t, nullptr);
  }
  return p;
}

// Scw decomposition (ORBmatcher.cc:308-312, :1006-1010): scw = sqrt(row0 . row0) with Mat::dot
// in double; sRcw / scw and col(3) / scw are MatExpr scalings evaluated by convertTo with the
// float factor (float)(1 / scw); Ow = -Rcw^T tcw.
Pose pose_from_sim3(const float* S) {
  double d = 0.0;
  for (int k = 0; k < 3; k++) d += (double)S[k] * (double)S[k];
  const float scw = (float)std::sqrt(d);
  const float a = (float)(1.0 / (double)scw);
  Pose p;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) p.R[3 * r + c] = S[4 * r + c] * a;
    p.t[r] = S[4 * r + 3] * a;
  }
  for (int i = 0; i < 3; i++) {
    const float col[3] = {p.R[i], p.R[3 + i], p.R[6 + i]};
    p.Ow[i] = -gemv_row(col, p.t, nullptr);
  }
  return p;
}

inline void transform(const float* R, const float* t, const float* X, float* out) {
  for (int r = 0; r < 3; r++) out[r] = gemv_row(R + 3 * r, X, &t[r]);
}

inline bool in_image_kf(const orbfe_frame_view* K, float u, float v) {  // KeyFrame.cc:627-630
  return u >= K->min_x && u < K->max_x && v >= K->min_y && v < K->max_y;
}

inline bool has_good_mp(uint8_t st) { return st != ORBFE_MP_NONE && st != ORBFE_MP_BAD; }

// rotation-consistency removal of ORBmatcher.cc:272-290 / :648-666 / :1603-1622
template <class Undo>
void rotation_filter(std::vector<int>* rotHist, int& nm, Undo undo) {
  int ind1 = -1, ind2 = -1, ind3 = -1;
  three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
  for (int b = 0; b < HISTO_LENGTH; b++) {
    if (b == ind1 || b == ind2 || b == ind3) continue;
    for (int j : rotHist[b]) {
      undo(j);
      nm--;
    }
  }
}

// The FeatureVector merge-join of :181-270 / :559-646: calls node(a, b) for every common node id.
template <class Node>
void merge_join(const orbfe_feature_vector* f1, const orbfe_feature_vector* f2, Node node) {
  int a = 0, b = 0;
  while (a < f1->n_nodes && b < f2->n_nodes) {
    const uint32_t id1 = f1->node_ids[a], id2 = f2->node_ids[b];
    if (id1 == id2) {
      node(a, b);
      a++;
      b++;
    } else if (id1 < id2) {
      a = (int)(std::lower_bound(f1->node_ids + a, f1->node_ids + f1->n_nodes, id2) - f1->node_ids);
    } else {
      b = (int)(std::lower_bound(f2->node_ids + b, f2->node_ids + f2->n_nodes, id1) - f2->node_ids);
    }
  }
}
}  // namespace

// SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (ORBmatcher.cc:165-293)
extern "C" int orbref_search_by_bow_kf_frame(const orbfe_frame_view* K, const orbfe_feature_vector* fk,
                                             const orbfe_frame_view* F, const orbfe_feature_vector* ff,
                                             float nnratio, int check_ori, int32_t* match_f,
                                             int* nmatches) {
  if (!K || !fk || !F || !ff || !nmatches || (F->n > 0 && !match_f)) return ORBFE_ERR_ARG;
  for (int k = 0; k < F->n; k++) match_f[k] = -1;  // vpMapPointMatches = NULL (:169)
  std::vector<int> rotHist[HISTO_LENGTH];
  int nm = 0;
  merge_join(fk, ff, [&](int a, int b) {
    for (int p = fk->offsets[a]; p < fk->offsets[a + 1]; p++) {
      const int realIdxKF = fk->indices[p];
      if (!has_good_mp(K->mp_state[realIdxKF])) continue;  // !pMP || isBad (:199-203)
      const uint8_t* dKF = K->descriptors + (size_t)realIdxKF * 32;
      int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
      for (int q = ff->offsets[b]; q < ff->offsets[b + 1]; q++) {
        const int realIdxF = ff->indices[q];
        if (match_f[realIdxF] >= 0) continue;  // vpMapPointMatches[realIdxF] (:215)
        const int dist = desc_distance(dKF, F->descriptors + (size_t)realIdxF * 32);
        if (dist < bestDist1) {
          bestDist2 = bestDist1;
          bestDist1 = dist;
          bestIdxF = realIdxF;
        } else if (dist < bestDist2) {
          bestDist2 = dist;
        }
      }
      if (bestDist1 <= TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {
        match_f[bestIdxF] = realIdxKF;
        if (check_ori) rotHist[rot_bin(K->keys_un[realIdxKF].angle, F->keys_un[bestIdxF].angle)].push_back(bestIdxF);
        nm++;
      }
    }
  });
  if (check_ori) rotation_filter(rotHist, nm, [&](int k) { match_f[k] = -1; });
  *nmatches = nm;
  return ORBFE_OK;
}

// SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (ORBmatcher.cc:536-669)
extern "C" int orbref_search_by_bow_kf_kf(const orbfe_frame_view* K1, const orbfe_feature_vector* f1,
                                          const orbfe_frame_view* K2, const orbfe_feature_vector* f2,
                                          float nnratio, int check_ori, int32_t* match12, int* nmatches) {
  if (!K1 || !f1 || !K2 || !f2 || !nmatches || (K1->n > 0 && !match12)) return ORBFE_ERR_ARG;
  for (int i = 0; i < K1->n; i++) match12[i] = -1;
  std::vector<uint8_t> matched2(K2->n, 0);
  std::vector<int> rotHist[HISTO_LENGTH];
  int nm = 0;
  merge_join(f1, f2, [&](int a, int b) {
    for (int p = f1->offsets[a]; p < f1->offsets[a + 1]; p++) {
      const int idx1 = f1->indices[p];
      if (!has_good_mp(K1->mp_state[idx1])) continue;  // :572-576
      const uint8_t* d1 = K1->descriptors + (size_t)idx1 * 32;
      int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
      for (int q = f2->offsets[b]; q < f2->offsets[b + 1]; q++) {
        const int idx2 = f2->indices[q];
        if (matched2[idx2] || !has_good_mp(K2->mp_state[idx2])) continue;  // :590-594
        const int dist = desc_distance(d1, K2->descriptors + (size_t)idx2 * 32);
        if (dist < bestDist1) {
          bestDist2 = bestDist1;
          bestDist1 = dist;
          bestIdx2 = idx2;
        } else if (dist < bestDist2) {
          bestDist2 = dist;
        }
      }
      if (bestDist1 < TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {
        match12[idx1] = bestIdx2;
        matched2[bestIdx2] = 1;
        if (check_ori) rotHist[rot_bin(K1->keys_un[idx1].angle, K2->keys_un[bestIdx2].angle)].push_back(idx1);
        nm++;
      }
    }
  });
  if (check_ori) rotation_filter(rotHist, nm, [&](int i) { match12[i] = -1; });
  *nmatches = nm;
  return ORBFE_OK;
}

// SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist) (ORBmatcher.cc:1493-1625)
extern "C" int orbref_search_by_projection_keyframe(const orbfe_frame_view* C, const float* Tcw,
                                                    const orbfe_mappoint_geometry* P,
                                                    const float* kf_angle, float log_scale_factor,
                                                    float th, int orb_dist, int check_ori,
                                                    int32_t* best_idx, int* nmatches) {
  if (!C || !Tcw || !P || !nmatches || (P->m > 0 && (!best_idx || !kf_angle))) return ORBFE_ERR_ARG;
  const Pose ps = pose_from(Tcw);
  const Grid g = build_grid(C);
  std::vector<uint8_t> blocked(C->n);
  for (int k = 0; k < C->n; k++) blocked[k] = C->mp_state[k] != ORBFE_MP_NONE;  // mvpMapPoints[i2] (:1567)
  std::vector<int> rotHist[HISTO_LENGTH];
  std::vector<int> idxs;
  int nm = 0;
  for (int i = 0; i < P->m; i++) {
    best_idx[i] = -1;
    const uint8_t fl = P->flags[i];
    if (!(fl & ORBFE_MPF_PRESENT) || (fl & (ORBFE_MPF_BAD | ORBFE_MPF_SKIP))) continue;  // :1517-1519
    const float* X = P->world_pos + 3 * (size_t)i;
    float Xc[3];
    transform(ps.R, ps.t, X, Xc);
    const float invzc = (float)(1.0 / (double)Xc[2]);
    const float u = C->fx * Xc[0] * invzc + C->cx;
    const float v = C->fy * Xc[1] * invzc + C->cy;
    if (u < C->min_x || u > C->max_x) continue;
    if (v < C->min_y || v > C->max_y) continue;
    const float PO[3] = {X[0] - ps.Ow[0], X[1] - ps.Ow[1], X[2] - ps.Ow[2]};
    const float dist3D = norm3(PO);
    const float maxDistance = 1.2f * P->max_distance[i];
    const float minDistance = 0.8f * P->min_distance[i];
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int pred = predict_scale(P->max_distance[i], dist3D, log_scale_factor, C->nlevels);
    const float radius = th * C->scale_factors[pred];
    features_in_area(C, g, u, v, radius, pred - 1, pred + 1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = P->descriptors + (size_t)i * 32;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : idxs) {
      if (blocked[i2]) continue;
      const int dist = desc_distance(dMP, C->descriptors + (size_t)i2 * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= orb_dist) {
      best_idx[i] = bestIdx2;
      blocked[bestIdx2] = 1;
      nm++;
      if (check_ori) rotHist[rot_bin(kf_angle[i], C->keys_un[bestIdx2].angle)].push_back(i);
    }
  }
  if (check_ori) rotation_filter(rotHist, nm, [&](int i) { best_idx[i] = -2 - best_idx[i]; });
  *nmatches = nm;
  return ORBFE_OK;
}

// SearchByProjection(KeyFrame*, cv::Mat Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:295-412)
extern "C" int orbref_search_by_projection_sim3(const orbfe_frame_view* K, const float* Scw,
                                                const orbfe_mappoint_geometry* P,
                                                float log_scale_factor, int th, int32_t* best_idx,
                                                int* nmatches) {
  if (!K || !Scw || !P || !nmatches || (P->m > 0 && !best_idx)) return ORBFE_ERR_ARG;
  const Pose ps = pose_from_sim3(Scw);
  const Grid g = build_grid(K);
  std::vector<uint8_t> taken(K->n);
  for (int k = 0; k < K->n; k++) taken[k] = K->mp_state[k] != ORBFE_MP_NONE;  // vpMatched[idx] (:384)
  std::vector<int> idxs;
  int nm = 0;
  for (int i = 0; i < P->m; i++) {
    best_idx[i] = -1;
    const uint8_t fl = P->flags[i];
    if (fl & (ORBFE_MPF_BAD | ORBFE_MPF_SKIP)) continue;  // :326
    const float* X = P->world_pos + 3 * (size_t)i;
    float Xc[3];
    transform(ps.R, ps.t, X, Xc);
    if (Xc[2] < 0.0) continue;
    const float invz = 1 / Xc[2];
    const float x = Xc[0] * invz, y = Xc[1] * invz;
    const float u = K->fx * x + K->cx, v = K->fy * y + K->cy;
    if (!in_image_kf(K, u, v)) continue;
    const float maxDistance = 1.2f * P->max_distance[i];
    const float minDistance = 0.8f * P->min_distance[i];
    const float PO[3] = {X[0] - ps.Ow[0], X[1] - ps.Ow[1], X[2] - ps.Ow[2]};
    const float dist = norm3(PO);
    if (dist < minDistance || dist > maxDistance) continue;
    if (dot3(PO, P->normal + 3 * (size_t)i) < 0.5 * dist) continue;
    const int pred = predict_scale(P->max_distance[i], dist, log_scale_factor, K->nlevels);
    const float radius = th * K->scale_factors[pred];
    features_in_area(K, g, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = P->descriptors + (size_t)i * 32;
    int bestDist = 256, bestIdx = -1;
    for (int idx : idxs) {
      if (taken[idx]) continue;
      const int kpLevel = K->keys_un[idx].octave;
      if (kpLevel < pred - 1 || kpLevel > pred) continue;
      const int d = desc_distance(dMP, K->descriptors + (size_t)idx * 32);
      if (d < bestDist) {
        bestDist = d;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_LOW) {
      best_idx[i] = bestIdx;
      taken[bestIdx] = 1;
      nm++;
    }
  }
  *nmatches = nm;
  return ORBFE_OK;
}

// Fuse(KeyFrame*, const vector<MapPoint*>&, th) (ORBmatcher.cc:841-991): the search part
extern "C" int orbref_fuse(const orbfe_frame_view* K, const float* Tcw, const float* Ow,
                           const orbfe_mappoint_geometry* P, float log_scale_factor, float th,
                           int32_t* best_idx, int* n_candidates) {
  if (!K || !Tcw || !Ow || !P || !n_candidates || (P->m > 0 && !best_idx) || !K->level_sigma2)
    return ORBFE_ERR_ARG;
  const Pose ps = pose_from(Tcw);
  const Grid g = build_grid(K);
  std::vector<float> invSigma2(K->nlevels);
  for (int l = 0; l < K->nlevels; l++) invSigma2[l] = 1.0f / K->level_sigma2[l];  // ORBextractor.cc:433
  std::vector<int> idxs;
  int n = 0;
  for (int i = 0; i < P->m; i++) {
    best_idx[i] = -1;
    const uint8_t fl = P->flags[i];
    if (!(fl & ORBFE_MPF_PRESENT) || (fl & (ORBFE_MPF_BAD | ORBFE_MPF_SKIP))) continue;  // :862-866
    const float* X = P->world_pos + 3 * (size_t)i;
    float Xc[3];
    transform(ps.R, ps.t, X, Xc);
    if (Xc[2] < 0.0f) continue;
    const float invz = 1 / Xc[2];
    const float x = Xc[0] * invz, y = Xc[1] * invz;
    const float u = K->fx * x + K->cx, v = K->fy * y + K->cy;
    if (!in_image_kf(K, u, v)) continue;
    const float ur = u - K->bf * invz;
    const float maxDistance = 1.2f * P->max_distance[i];
    const float minDistance = 0.8f * P->min_distance[i];
    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
    const float dist3D = norm3(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    if (dot3(PO, P->normal + 3 * (size_t)i) < 0.5 * dist3D) continue;
    const int pred = predict_scale(P->max_distance[i], dist3D, log_scale_factor, K->nlevels);
    const float radius = th * K->scale_factors[pred];
    features_in_area(K, g, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = P->descriptors + (size_t)i * 32;
    int bestDist = 256, bestIdx = -1;
    for (int idx : idxs) {
      const orbfe_keypoint& kp = K->keys_un[idx];
      const int kpLevel = kp.octave;
      if (kpLevel < pred - 1 || kpLevel > pred) continue;
      if (K->u_right[idx] >= 0) {
        const float ex = u - kp.x, ey = v - kp.y, er = ur - K->u_right[idx];
        const float e2 = ex * ex + ey * ey + er * er;
        if (e2 * invSigma2[kpLevel] > 7.8) continue;
      } else {
        const float ex = u - kp.x, ey = v - kp.y;
        const float e2 = ex * ex + ey * ey;
        if (e2 * invSigma2[kpLevel] > 5.99) continue;
      }
      const int d = desc_distance(dMP, K->descriptors + (size_t)idx * 32);
      if (d < bestDist) {
        bestDist = d;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_LOW) {
      best_idx[i] = bestIdx;
      n++;
    }
  }
  *n_candidates = n;
  return ORBFE_OK;
}

// Fuse(KeyFrame*, cv::Mat Scw, vpPoints, th, vpReplacePoint) (ORBmatcher.cc:993-1120): the search
extern "C" int orbref_fuse_sim3(const orbfe_frame_view* K, const float* Scw,
                                const orbfe_mappoint_geometry* P, float log_scale_factor, float th,
                                int32_t* best_idx, int* nfused) {
  if (!K || !Scw || !P || !nfused || (P->m > 0 && !best_idx)) return ORBFE_ERR_ARG;
  const Pose ps = pose_from_sim3(Scw);
  const Grid g = build_grid(K);
  std::vector<int> idxs;
  int n = 0;
  for (int i = 0; i < P->m; i++) {
    best_idx[i] = -1;
    const uint8_t fl = P->flags[i];
    if (fl & (ORBFE_MPF_BAD | ORBFE_MPF_SKIP)) continue;  // :1025
    const float* X = P->world_pos + 3 * (size_t)i;
    float Xc[3];
    transform(ps.R, ps.t, X, Xc);
    if (Xc[2] < 0.0f) continue;
    const float invz = (float)(1.0 / (double)Xc[2]);
    const float x = Xc[0] * invz, y = Xc[1] * invz;
    const float u = K->fx * x + K->cx, v = K->fy * y + K->cy;
    if (!in_image_kf(K, u, v)) continue;
    const float maxDistance = 1.2f * P->max_distance[i];
    const float minDistance = 0.8f * P->min_distance[i];
    const float PO[3] = {X[0] - ps.Ow[0], X[1] - ps.Ow[1], X[2] - ps.Ow[2]};
    const float dist3D = norm3(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    if (dot3(PO, P->normal + 3 * (size_t)i) < 0.5 * dist3D) continue;
    const int pred = predict_scale(P->max_distance[i], dist3D, log_scale_factor, K->nlevels);
    const float radius = th * K->scale_factors[pred];
    features_in_area(K, g, u, v, radius, -1, -1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* dMP = P->descriptors + (size_t)i * 32;
    int bestDist = INT_MAX, bestIdx = -1;
    for (int idx : idxs) {
      const int kpLevel = K->keys_un[idx].octave;
      if (kpLevel < pred - 1 || kpLevel > pred) continue;
      const int d = desc_distance(dMP, K->descriptors + (size_t)idx * 32);
      if (d < bestDist) {
        bestDist = d;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_LOW) {
      best_idx[i] = bestIdx;
      n++;
    }
  }
  *nfused = n;
  return ORBFE_OK;
}

// SearchBySim3(KF1, KF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1122-1346)
extern "C" int orbref_search_by_sim3(const orbfe_frame_view* K1, const orbfe_frame_view* K2,
                                     const orbfe_mappoint_geometry* M1, const orbfe_mappoint_geometry* M2,
                                     const float* T1w, const float* T2w, float s12, const float* R12,
                                     const float* t12, float lsf1, float lsf2, float th,
                                     int32_t* match12, int* nfound) {
  if (!K1 || !K2 || !M1 || !M2 || !T1w || !T2w || !R12 || !t12 || !nfound || (K1->n > 0 && !match12) ||
      M1->m != K1->n || M2->m != K2->n)
    return ORBFE_ERR_ARG;
  const Pose p1 = pose_from(T1w), p2 = pose_from(T2w);
  float sR12[9], sR21[9], t21[3];
  const float inv_s = (float)(1.0 / (double)s12);  // (1.0 / s12) * R12.t() (:1140)
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      sR12[3 * r + c] = R12[3 * r + c] * s12;  // s12 * R12 (:1139)
      sR21[3 * r + c] = R12[3 * c + r] * inv_s;
    }
  for (int r = 0; r < 3; r++) t21[r] = -gemv_row(sR21 + 3 * r, t12, nullptr);  // -sR21 * t12 (:1141)
  const Grid g1 = build_grid(K1), g2 = build_grid(K2);
  std::vector<int> vnMatch1(K1->n, -1), vnMatch2(K2->n, -1), idxs;
  // one direction: MapPoints of KA projected into KB (camera of K1, as the reference)
  auto search = [&](const orbfe_frame_view* KB, const Grid& gB, const orbfe_mappoint_geometry* MA,
                    const Pose& pA, const float* sR, const float* tt, float lsfB, std::vector<int>& out) {
    for (int i = 0; i < MA->m; i++) {
      const uint8_t fl = MA->flags[i];
      if (!(fl & ORBFE_MPF_PRESENT) || (fl & ORBFE_MPF_SKIP)) continue;  // :1172 / :1252
      if (fl & ORBFE_MPF_BAD) continue;
      const float* X = MA->world_pos + 3 * (size_t)i;
      float Xa[3], Xb[3];
      transform(pA.R, pA.t, X, Xa);
      transform(sR, tt, Xa, Xb);
      if (Xb[2] < 0.0) continue;
      const float invz = (float)(1.0 / (double)Xb[2]);
      const float x = Xb[0] * invz, y = Xb[1] * invz;
      const float u = K1->fx * x + K1->cx, v = K1->fy * y + K1->cy;
      if (!in_image_kf(KB, u, v)) continue;
      const float maxDistance = 1.2f * MA->max_distance[i];
      const float minDistance = 0.8f * MA->min_distance[i];
      const float dist3D = norm3(Xb);
      if (dist3D < minDistance || dist3D > maxDistance) continue;
      const int pred = predict_scale(MA->max_distance[i], dist3D, lsfB, KB->nlevels);
      const float radius = th * KB->scale_factors[pred];
      features_in_area(KB, gB, u, v, radius, -1, -1, idxs);
      if (idxs.empty()) continue;
      const uint8_t* dMP = MA->descriptors + (size_t)i * 32;
      int bestDist = INT_MAX, bestIdx = -1;
      for (int idx : idxs) {
        const int oct = KB->keys_un[idx].octave;
        if (oct < pred - 1 || oct > pred) continue;
        const int d = desc_distance(dMP, KB->descriptors + (size_t)idx * 32);
        if (d < bestDist) {
          bestDist = d;
          bestIdx = idx;
        }
      }
      if (bestDist <= TH_HIGH) out[i] = bestIdx;
    }
  };
  search(K2, g2, M1, p1, sR21, t21, lsf2, vnMatch1);
  search(K1, g1, M2, p2, sR12, t12, lsf1, vnMatch2);
  int n = 0;
  for (int i1 = 0; i1 < K1->n; i1++) {  // check agreement (:1328-1343)
    match12[i1] = -1;
    const int idx2 = vnMatch1[i1];
    if (idx2 >= 0 && vnMatch2[idx2] == i1) {
      match12[i1] = idx2;
      n++;
    }
  }
  *nfound = n;
  return ORBFE_OK;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:414-534)
extern "C" int orbref_search_for_initialization(const orbfe_frame_view* F1, const orbfe_frame_view* F2,
                                                float* prev, int window, float nnratio, int check_ori,
                                                int32_t* match12, int* nmatches) {
  if (!F1 || !F2 || !nmatches || (F1->n > 0 && (!prev || !match12))) return ORBFE_ERR_ARG;
  const Grid g2 = build_grid(F2);
  for (int i = 0; i < F1->n; i++) match12[i] = -1;
  std::vector<int> vMatchedDistance(F2->n, INT_MAX), vnMatches21(F2->n, -1), idxs;
  std::vector<int> rotHist[HISTO_LENGTH];
  int nm = 0;
  for (int i1 = 0; i1 < F1->n; i1++) {
    const int level1 = F1->keys_un[i1].octave;
    if (level1 > 0) continue;
    features_in_area(F2, g2, prev[2 * i1], prev[2 * i1 + 1], (float)window, level1, level1, idxs);
    if (idxs.empty()) continue;
    const uint8_t* d1 = F1->descriptors + (size_t)i1 * 32;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (int i2 : idxs) {
      const int dist = desc_distance(d1, F2->descriptors + (size_t)i2 * 32);
      if (vMatchedDistance[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_LOW && (float)bestDist < (float)bestDist2 * nnratio) {
      if (vnMatches21[bestIdx2] >= 0) {
        match12[vnMatches21[bestIdx2]] = -1;
        nm--;
      }
      match12[i1] = bestIdx2;
      vnMatches21[bestIdx2] = i1;
      vMatchedDistance[bestIdx2] = bestDist;
      nm++;
      if (check_ori) rotHist[rot_bin(F1->keys_un[i1].angle, F2->keys_un[bestIdx2].angle)].push_back(i1);
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int b = 0; b < HISTO_LENGTH; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int idx1 : rotHist[b])
        if (match12[idx1] >= 0) {
          match12[idx1] = -1;
          nm--;
        }
    }
  }
  for (int i1 = 0; i1 < F1->n; i1++)  // update prev matched (:528-531)
    if (match12[i1] >= 0) {
      prev[2 * i1] = F2->keys_un[match12[i1]].x;
      prev[2 * i1 + 1] = F2->keys_un[match12[i1]].y;
    }
  *nmatches = nm;
  return ORBFE_OK;
}

// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:272-337): BestIdx per MapPoint
extern "C" int orbref_compute_distinctive_descriptors(int n_points, const int32_t* offsets,
                                                      const uint8_t* desc, int32_t* best_index) {
  if (n_points < 0 || (n_points > 0 && (!offsets || !best_index))) return ORBFE_ERR_ARG;
  for (int p = 0; p < n_points; p++) {
    const int o = offsets[p];
    const size_t N = (size_t)(offsets[p + 1] - o);
    if (N == 0) {  // vDescriptors.empty(): return (:299-300)
      best_index[p] = -1;
      continue;
    }
    std::vector<float> D(N * N);
    for (size_t i = 0; i < N; i++) {
      D[i * N + i] = 0;
      for (size_t j = i + 1; j < N; j++) {
        const int d = desc_distance(desc + 32 * (size_t)(o + i), desc + 32 * (size_t)(o + j));
        D[i * N + j] = (float)d;
        D[j * N + i] = (float)d;
      }
    }
    int BestMedian = INT_MAX, BestIdx = 0;
    std::vector<int> row(N);
    for (size_t i = 0; i < N; i++) {
      for (size_t j = 0; j < N; j++) row[j] = (int)D[i * N + j];
      std::sort(row.begin(), row.end());
      const int median = row[(size_t)(0.5 * (N - 1))];
      if (median < BestMedian) {
        BestMedian = median;
        BestIdx = (int)i;
      }
    }
    best_index[p] = BestIdx;
  }
  return ORBFE_OK;
}

// Exhaustive check of a PredictScale threshold table (orbfe_predict_scale_thresholds) against the
// reference formula over every float ratio with bit pattern in [lo_bits, hi_bits]: returns the
// number of ratios where #{k : ratio >= thr[k-1]} differs from clamp(ceil(logf(r) / lsf)), and
// (in *non_monotone) how many times the reference formula decreased between neighbouring floats.
extern "C" long long orbref_check_predict_scale(float lsf, int nlevels, const float* thr, uint32_t lo_bits,
                                                uint32_t hi_bits, long long* non_monotone) {
  long long bad = 0, nm = 0;
  int last = INT_MIN;
  for (uint64_t b = lo_bits; b <= hi_bits; b++) {
    const uint32_t bits = (uint32_t)b;
    float r;
    std::memcpy(&r, &bits, 4);
    const int raw = (int)std::ceil(std::log(r) / lsf);  // MapPoint.cc:424 (float overloads)
    const int want = raw < 0 ? 0 : (raw >= nlevels ? nlevels - 1 : raw);
    int got = 0;
    for (int k = 1; k < nlevels; k++) got += r >= thr[k - 1];
    bad += got != want;
    if (raw < last) nm++;
    last = raw;
  }
  if (non_monotone) *non_monotone = nm;
  return bad;
}
