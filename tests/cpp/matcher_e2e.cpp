// The matcher half of the drop-in: adapter/ORBmatcher_gpu.cc compiled over the test-only reference
// declarations (tests/cpp/cvstub: Frame, KeyFrame, MapPoint, ORBmatcher, DBoW2) and run on the GPU
// the way the reference's threads call it, on a stereo driving sequence (orbfe_synth_sequence_frame:
// frames 1 m apart along z) whose MapPoints are triangulated from the stereo matches:
//   Tracking::TrackWithMotionModel (Tracking.cc:889-915): SearchByProjection(CurrentFrame,
//     LastFrame, th, bMono) with th 7 (stereo) and the 2*th retry below 20 matches, taken and not
//     taken, and th 15 mono;
//   Tracking::SearchLocalPoints (:1186-1214): isInFrustum (the oracle's, standing in for
//     Frame::isInFrustum, which is not on the adapter) then SearchByProjection(F, vpLocalMapPoints,
//     th) with th 1 and 5;
//   LocalMapping::CreateNewMapPoints (LocalMapping.cc:219-272): SearchForTriangulation(pKF1, pKF2,
//     F12, vMatchedPairs, bOnlyStereo), the epipole computed inside the adapter (ORBmatcher.cc:678-684);
//   Tracking::Relocalization (:1459-1495): SearchByBoW(pKF, F, vpMapPointMatches), then
//     SearchByProjection(F, pKF, sFound, 10, 100) after a stand-in for the PnP inliers;
//   LoopClosing::ComputeSim3 (LoopClosing.cc:402): SearchByProjection(pKF, Scw, vpPoints,
//     vpMatched, 10).
// Each call's expected result comes from the CPU oracle (oracle/orbref.h, test infrastructure) on
// views this file packs itself from the objects, applied with the reference's own loop
// (ORBmatcher.cc:127, :1434-1488, :828-836, :283-286, :1616-1620, :404-406); every applied
// mvpMapPoints / vpMapPointMatches / vpMatched entry and every vMatchedPairs entry is compared.
// Prints one "MATCHER {json}" line, then OK / MISMATCH. Exit: 0 parity ok, 1 mismatch, 77 no GPU.
// `matcher_e2e --dry` builds the scene and runs only the oracle side (CPU; the scenario checks, e.g.
// that the retry case takes the retry, still apply).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "ORBmatcher.h"
#include "orbfe.hpp"
#include "orbfe_synth.h"
#include "../../oracle/orbref.h"

using namespace ORB_SLAM2;

// the checker reads the protected scale-invariance distances as the reference's ORBmatcher does
struct orbfe_test_access {
  static void dist(MapPoint* p, float& dmin, float& dmax) {
    std::lock_guard<std::mutex> lock(p->mMutexPos);
    dmin = p->mfMinDistance;
    dmax = p->mfMaxDistance;
  }
};

namespace {
constexpr int kRows = 376, kCols = 1241, kLevels = 8;
constexpr float kFx = 718.856f, kCx = 607.1928f, kCy = 185.2157f, kBf = 386.1448f;
constexpr uint64_t kSeqSeed = 0x5EC0E2Eull;

int g_fails = 0;
bool g_dry = false;  // --dry: the oracle side only (no device)
void fail(const std::string& what) {
  std::printf("MISMATCH %s\n", what.c_str());
  g_fails++;
}

// ---- scene --------------------------------------------------------------------------------------
cv::Mat pose_z(float tz, float yaw = 0.f) {  // Tcw = [Ry(yaw) | Ry(yaw) * (0, 0, -tz)]
  cv::Mat T = cv::Mat::eye(4, 4, CV_32F);
  const float c = std::cos(yaw), s = std::sin(yaw);
  T.at<float>(0, 0) = c;
  T.at<float>(0, 2) = s;
  T.at<float>(2, 0) = -s;
  T.at<float>(2, 2) = c;
  T.at<float>(0, 3) = -s * tz;
  T.at<float>(2, 3) = -c * tz;
  return T;
}

struct Vocab {
  orbref_vocab* v = nullptr;
  ~Vocab() { orbref_vocab_free(v); }
};

// a k = 10, L = 2 DBoW2 tree whose node descriptors are descriptors of the scene's first frame
void build_vocab(const cv::Mat& desc, Vocab& voc) {
  const int k = 10, n_nodes = 1 + k + k * k;
  std::vector<int32_t> parent(n_nodes, -1);
  std::vector<uint8_t> is_leaf(n_nodes, 0), nd((size_t)n_nodes * 32, 0);
  std::vector<double> w(n_nodes, 1.0);
  for (int i = 1; i < n_nodes; i++) {
    parent[i] = i <= k ? 0 : 1 + (i - 1 - k) / k;
    is_leaf[i] = i > k;
    std::memcpy(&nd[(size_t)i * 32], desc.ptr<uint8_t>((i * 37) % desc.rows), 32);
  }
  if (orbref_vocab_from_table(n_nodes, k, 2, 0, 0, parent.data(), is_leaf.data(), nd.data(), w.data(), &voc.v))
    throw std::runtime_error("vocabulary");
}

// KeyFrame::ComputeBoW's FeatureVector (levelsup 1 on this L = 2 tree: the level-1 nodes)
DBoW2::FeatureVector feature_vector(const Vocab& voc, const cv::Mat& desc) {
  const int n = desc.rows;
  std::vector<uint32_t> words(n + 1), ids(n + 1);
  std::vector<double> wts(n + 1);
  std::vector<int32_t> off(n + 2), idx(n + 1);
  int nw = 0, nn = 0;
  orbref_vocab_transform_full(voc.v, desc.data, n, 1, words.data(), wts.data(), &nw, ids.data(), off.data(),
                              idx.data(), &nn);
  DBoW2::FeatureVector fv;
  for (int j = 0; j < nn; j++)
    for (int q = off[j]; q < off[j + 1]; q++) fv.addFeature(ids[j], (unsigned)idx[q]);
  return fv;
}

struct Extracted {
  std::vector<orbfe_keypoint> k;
  std::vector<uint8_t> d;
  std::vector<std::vector<uint8_t>> lv;
  int rows[kLevels], cols[kLevels];
};

Extracted oracle_extract(const std::vector<uint8_t>& img) {
  Extracted r;
  orbref_extractor* e = orbref_extractor_create(2000, 1.2f, kLevels, 20, 7);
  const int cap = 8000;
  r.k.resize(cap);
  r.d.resize((size_t)cap * 32);
  int n = 0;
  orbref_extract(e, img.data(), kRows, kCols, kCols, r.k.data(), cap, r.d.data(), &n);
  r.k.resize(n);
  r.d.resize((size_t)n * 32);
  r.lv.resize(kLevels);
  for (int l = 0; l < kLevels; l++) {
    orbref_get_level(e, l, nullptr, 0, &r.rows[l], &r.cols[l]);
    r.lv[l].resize((size_t)r.rows[l] * r.cols[l]);
    orbref_get_level(e, l, r.lv[l].data(), (int)r.lv[l].size(), &r.rows[l], &r.cols[l]);
  }
  orbref_extractor_destroy(e);
  return r;
}

// the stereo Frame of sequence frame t (Frame.cc:94-160 for a rectified pair): keypoints and
// descriptors of both images, ComputeStereoMatches, the scale tables and the true pose
void make_frame(long long t, Frame& F) {
  std::vector<uint8_t> L((size_t)kRows * kCols), R((size_t)kRows * kCols);
  if (orbfe_synth_sequence_frame(kSeqSeed, t, kRows, kCols, kFx, kFx, kCx, kCy, kBf / kFx, 1.0f, L.data(), R.data(),
                                 kCols))
    throw std::runtime_error("synth");
  const Extracted el = oracle_extract(L), er = oracle_extract(R);
  orbref_extractor* e = orbref_extractor_create(2000, 1.2f, kLevels, 20, 7);
  std::vector<float> scale(kLevels), inv(kLevels), s2(kLevels), is2(kLevels);
  std::vector<int32_t> fpl(kLevels), umax(16);
  orbref_get_tables(e, scale.data(), inv.data(), s2.data(), is2.data(), fpl.data(), umax.data());
  orbref_extractor_destroy(e);
  orbref_level_view vl[kLevels], vr[kLevels];
  for (int l = 0; l < kLevels; l++) {
    vl[l] = orbref_level_view{el.lv[l].data(), el.rows[l], el.cols[l], el.cols[l]};
    vr[l] = orbref_level_view{er.lv[l].data(), er.rows[l], er.cols[l], er.cols[l]};
  }
  const int n = (int)el.k.size();
  F.N = n;
  F.mvKeys.resize(n);
  for (int i = 0; i < n; i++) {
    const orbfe_keypoint& k = el.k[i];
    F.mvKeys[i] = cv::KeyPoint(k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id);
  }
  F.mvKeysUn = F.mvKeys;  // rectified KITTI-shaped input: no distortion
  F.mvuRight.assign(n, -1.f);
  F.mvDepth.assign(n, -1.f);
  orbref_compute_stereo_matches(el.k.data(), el.d.data(), n, er.k.data(), er.d.data(), (int)er.k.size(), vl, vr,
                                kLevels, scale.data(), inv.data(), kBf / kFx, kBf, F.mvuRight.data(), F.mvDepth.data());
  F.mDescriptors = cv::Mat(n, 32, CV_8U);
  std::memcpy(F.mDescriptors.data, el.d.data(), el.d.size());
  F.mvpMapPoints.assign(n, nullptr);
  F.mvbOutlier.assign(n, false);
  F.mnScaleLevels = kLevels;
  F.mfScaleFactor = 1.2f;
  F.mfLogScaleFactor = std::log(F.mfScaleFactor);
  F.mvScaleFactors = scale;
  F.mvInvScaleFactors = inv;
  F.mvLevelSigma2 = s2;
  F.mvInvLevelSigma2 = is2;
  F.mbf = kBf;
  F.mb = kBf / kFx;
  F.mTcw = pose_z((float)t);
}

// Tracking::StereoInitialization / CreateNewKeyFrame's MapPoints (Tracking.cc:639-660): one per
// keypoint with a stereo depth, world position Twc * (x, y, z)
void add_stereo_mappoints(Frame& F, KeyFrame* kf, std::vector<std::unique_ptr<MapPoint>>& pool, int every) {
  const cv::Mat Twc = kf->GetPoseInverse();
  for (int i = 0; i < F.N; i += every) {
    const float z = F.mvDepth[i];
    if (z <= 0.f) continue;
    const float u = F.mvKeysUn[i].pt.x, v = F.mvKeysUn[i].pt.y;
    const float xc[3] = {(u - Frame::cx) * z / Frame::fx, (v - Frame::cy) * z / Frame::fy, z};
    cv::Mat X(3, 1, CV_32F);
    for (int r = 0; r < 3; r++)
      X.at<float>(r) = Twc.at<float>(r, 0) * xc[0] + Twc.at<float>(r, 1) * xc[1] + Twc.at<float>(r, 2) * xc[2] +
                       Twc.at<float>(r, 3);
    pool.emplace_back(new MapPoint(X, kf, nullptr));
    MapPoint* p = pool.back().get();
    p->AddObservation(kf, i);
    kf->AddMapPoint(p, i);
    p->ComputeDistinctiveDescriptors();
    p->UpdateNormalAndDepth();
    F.mvpMapPoints[i] = p;
  }
}

// ---- the checker's own packing of the objects (not adapter/orbfe_pack.hpp) -----------------------
struct View {
  std::vector<orbfe_keypoint> keys;
  std::vector<uint8_t> state;
  std::vector<float> u_right, scale, sigma2;
  std::vector<uint8_t> desc;
  orbfe_frame_view v{};
};

template <class FR>
void view_common(const FR& f, const std::vector<MapPoint*>& mps, bool keyframe, View& o) {
  o.keys.resize(f.N);
  for (int i = 0; i < f.N; i++) {
    const cv::KeyPoint& k = f.mvKeysUn[i];
    o.keys[i] = orbfe_keypoint{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave, k.class_id};
  }
  o.state.assign(f.N, ORBFE_MP_NONE);
  for (int i = 0; i < f.N; i++)
    if (MapPoint* p = mps[i])
      o.state[i] = keyframe && p->isBad() ? ORBFE_MP_BAD : p->Observations() > 0 ? ORBFE_MP_OBSERVED : ORBFE_MP_PRESENT;
  o.u_right = f.mvuRight;
  o.scale = f.mvScaleFactors;
  o.sigma2 = f.mvLevelSigma2;
  o.desc.assign(f.mDescriptors.data, f.mDescriptors.data + (size_t)f.N * 32);
  o.v = orbfe_frame_view{};
  o.v.n = f.N;
  o.v.keys_un = o.keys.data();
  o.v.u_right = o.u_right.data();
  o.v.descriptors = o.desc.data();
  o.v.mp_state = o.state.data();
  o.v.nlevels = f.mnScaleLevels;
  o.v.scale_factors = o.scale.data();
  o.v.level_sigma2 = o.sigma2.data();
  o.v.fx = Frame::fx;
  o.v.fy = Frame::fy;
  o.v.cx = Frame::cx;
  o.v.cy = Frame::cy;
  o.v.bf = f.mbf;
  o.v.b = f.mb;
  o.v.grid_inv_w = Frame::mfGridElementWidthInv;
  o.v.grid_inv_h = Frame::mfGridElementHeightInv;
}
void frame_view(const Frame& f, View& o) {
  view_common(f, f.mvpMapPoints, false, o);
  o.v.min_x = Frame::mnMinX;
  o.v.max_x = Frame::mnMaxX;
  o.v.min_y = Frame::mnMinY;
  o.v.max_y = Frame::mnMaxY;
}
void keyframe_view(KeyFrame* k, View& o) {
  view_common(*k, k->GetMapPointMatches(), true, o);
  o.v.min_x = (float)k->mnMinX;  // KeyFrame.h:202-205 keeps int bounds; its grid is the Frame's
  o.v.max_x = (float)k->mnMaxX;
  o.v.min_y = (float)k->mnMinY;
  o.v.max_y = (float)k->mnMaxY;
  o.v.grid_origin_set = 1;
  o.v.grid_min_x = Frame::mnMinX;
  o.v.grid_min_y = Frame::mnMinY;
}

struct Csr {
  std::vector<uint32_t> ids;
  std::vector<int32_t> off{0}, idx;
  orbfe_feature_vector v{};
  explicit Csr(const DBoW2::FeatureVector& fv) {
    for (const auto& kv : fv) {
      ids.push_back(kv.first);
      for (unsigned i : kv.second) idx.push_back((int32_t)i);
      off.push_back((int32_t)idx.size());
    }
    v = orbfe_feature_vector{(int32_t)ids.size(), ids.data(), off.data(), idx.data()};
  }
};

struct Geometry {  // MapPoint set -> orbfe_mappoint_geometry with the given flags
  std::vector<uint8_t> flags, desc;
  std::vector<float> pos, nrm, dmin, dmax;
  orbfe_mappoint_geometry v{};
  Geometry(const std::vector<MapPoint*>& mps, const std::vector<uint8_t>& fl) : flags(fl) {
    const size_t m = mps.size();
    desc.assign(m * 32, 0);
    pos.assign(m * 3, 0.f);
    nrm.assign(m * 3, 0.f);
    dmin.assign(m, 0.f);
    dmax.assign(m, 0.f);
    for (size_t i = 0; i < m; i++) {
      MapPoint* p = mps[i];
      if (!p) continue;
      const cv::Mat w = p->GetWorldPos(), n = p->GetNormal(), d = p->GetDescriptor();
      std::memcpy(&pos[i * 3], w.data, 12);
      std::memcpy(&nrm[i * 3], n.data, 12);
      std::memcpy(&desc[i * 32], d.data, 32);
      orbfe_test_access::dist(p, dmin[i], dmax[i]);
    }
    v = orbfe_mappoint_geometry{(int32_t)m, flags.data(), pos.data(), nrm.data(), dmin.data(), dmax.data(), desc.data()};
  }
};

// ---- the reference's result loops ---------------------------------------------------------------
void apply_local(const std::vector<int32_t>& best, std::vector<MapPoint*>& f, const std::vector<MapPoint*>& mps) {
  for (size_t i = 0; i < best.size(); i++)  // ORBmatcher.cc:127
    if (best[i] >= 0) f[best[i]] = mps[i];
}
void apply_with_rotation(const std::vector<int32_t>& best, std::vector<MapPoint*>& f, const std::vector<MapPoint*>& src) {
  for (size_t i = 0; i < best.size(); i++)  // the loop's assignments, then the rotation filter's NULLs
    if (best[i] >= 0 || best[i] <= -2) f[best[i] >= 0 ? best[i] : -2 - best[i]] = src[i];
  for (size_t i = 0; i < best.size(); i++)
    if (best[i] <= -2) f[-2 - best[i]] = nullptr;
}

void same_pointers(const std::vector<MapPoint*>& got, const std::vector<MapPoint*>& want, const std::string& tag) {
  if (got.size() != want.size()) return fail(tag + ": sizes differ");
  for (size_t i = 0; i < got.size(); i++)
    if (got[i] != want[i]) return fail(tag + ": entry " + std::to_string(i) + " differs");
}
int count_set(const std::vector<MapPoint*>& v) {
  int n = 0;
  for (MapPoint* p : v) n += p != nullptr;
  return n;
}

// ---- Tracking::TrackWithMotionModel's two calls (Tracking.cc:897-912) ---------------------------
struct MotionResult {
  int nmatches = 0;
  bool retried = false;
  std::vector<MapPoint*> mps;
};

MotionResult motion_expected(const Frame& cur, const Frame& last, float th, bool mono) {
  // LastFrame -> orbfe_lastframe_mappoints
  const int n = last.N;
  std::vector<uint8_t> flags(n, 0), desc((size_t)n * 32, 0);
  std::vector<float> pos((size_t)n * 3, 0.f), angle(n);
  std::vector<int32_t> octave(n);
  for (int i = 0; i < n; i++) {
    octave[i] = last.mvKeys[i].octave;
    angle[i] = last.mvKeysUn[i].angle;
    MapPoint* p = last.mvpMapPoints[i];
    if (!p) continue;
    flags[i] = ORBFE_MPF_PRESENT | (last.mvbOutlier[i] ? ORBFE_MPF_OUTLIER : 0u) |
               (p->Observations() > 0 ? ORBFE_MPF_OBSERVED : 0u);
    const cv::Mat w = p->GetWorldPos(), d = p->GetDescriptor();
    std::memcpy(&pos[(size_t)i * 3], w.data, 12);
    std::memcpy(&desc[(size_t)i * 32], d.data, 32);
  }
  orbfe_lastframe_mappoints lv{};
  lv.n = n;
  lv.flags = flags.data();
  lv.world_pos = pos.data();
  lv.descriptors = desc.data();
  lv.octave = octave.data();
  lv.angle = angle.data();
  std::memcpy(lv.tcw_last, last.mTcw.data, 12 * sizeof(float));
  MotionResult r;
  for (int pass = 0; pass < 2; pass++) {
    Frame c;  // fill(mvpMapPoints, NULL) before each call
    c.N = cur.N;
    c.mvKeysUn = cur.mvKeysUn;
    c.mvuRight = cur.mvuRight;
    c.mDescriptors = cur.mDescriptors;
    c.mvpMapPoints.assign(cur.N, nullptr);
    c.mnScaleLevels = cur.mnScaleLevels;
    c.mvScaleFactors = cur.mvScaleFactors;
    c.mvLevelSigma2 = cur.mvLevelSigma2;
    c.mbf = cur.mbf;
    c.mb = cur.mb;
    View cv_;
    frame_view(c, cv_);
    std::vector<int32_t> best(n, -1);
    const float t = pass == 0 ? th : 2 * th;
    orbref_search_by_projection_lastframe(&cv_.v, &lv, cur.mTcw.ptr<float>(), t, mono ? 1 : 0, 1, best.data(),
                                          &r.nmatches);
    apply_with_rotation(best, c.mvpMapPoints, last.mvpMapPoints);
    r.mps = c.mvpMapPoints;
    if (r.nmatches >= 20) break;
    r.retried = pass == 0;
  }
  return r;
}

MotionResult motion_adapter(Frame& cur, const Frame& last, float th, bool mono) {
  ORBmatcher matcher(0.9, true);  // Tracking.cc:889
  MotionResult r;
  std::fill(cur.mvpMapPoints.begin(), cur.mvpMapPoints.end(), static_cast<MapPoint*>(nullptr));
  r.nmatches = matcher.SearchByProjection(cur, last, th, mono);
  if (r.nmatches < 20) {
    r.retried = true;
    std::fill(cur.mvpMapPoints.begin(), cur.mvpMapPoints.end(), static_cast<MapPoint*>(nullptr));
    r.nmatches = matcher.SearchByProjection(cur, last, 2 * th, mono);
  }
  r.mps = cur.mvpMapPoints;
  return r;
}

std::string fmt_motion(const char* name, const MotionResult& r) {
  char b[160];
  std::snprintf(b, sizeof b, "\"%s\": {\"nmatches\": %d, \"retried\": %s, \"assigned\": %d}", name, r.nmatches,
                r.retried ? "true" : "false", count_set(r.mps));
  return b;
}
}  // namespace

int main(int argc, char** argv) {
  g_dry = argc > 1 && std::strcmp(argv[1], "--dry") == 0;
  if (!g_dry) try {
      orbfe::Matcher probe;  // the device check before anything else
    } catch (const orbfe::Error& e) {
      std::printf("no device: %s\n", e.what());
      return 77;
    }
  Frame::fx = Frame::fy = kFx;
  Frame::cx = kCx;
  Frame::cy = kCy;
  Frame::mnMinX = 0.f;
  Frame::mnMaxX = (float)kCols;
  Frame::mnMinY = 0.f;
  Frame::mnMaxY = (float)kRows;
  Frame::mfGridElementWidthInv = 64.f / (Frame::mnMaxX - Frame::mnMinX);  // FRAME_GRID_COLS / width
  Frame::mfGridElementHeightInv = 48.f / (Frame::mnMaxY - Frame::mnMinY);

  std::vector<std::unique_ptr<MapPoint>> pool;
  Frame F0, F1, F2;
  make_frame(0, F0);
  make_frame(1, F1);
  make_frame(2, F2);
  Vocab voc;
  build_vocab(F0.mDescriptors, voc);
  for (Frame* f : {&F0, &F1, &F2}) f->mFeatVec = feature_vector(voc, f->mDescriptors);

  // KeyFrame 0 with its stereo MapPoints; LastFrame = frame 0 with a few outliers
  KeyFrame K0(F0, nullptr, nullptr);
  add_stereo_mappoints(F0, &K0, pool, 1);
  for (int i = 0; i < F0.N; i += 13)
    if (F0.mvpMapPoints[i]) F0.mvbOutlier[i] = true;
  // a sparse last frame (every 12th MapPoint) for the retry case
  Frame F0s = F0;
  for (int i = 0; i < F0s.N; i++)
    if (i % 12) F0s.mvpMapPoints[i] = nullptr;

  std::string js;
  // ---- TrackWithMotionModel --------------------------------------------------------------------
  struct Case {
    const char* name;
    const Frame* last;
    float yaw, th;
    bool mono;
  };
  const Case cases[] = {{"motion_stereo_th7", &F0, 0.f, 7.f, false},
                        {"motion_stereo_retry", &F0s, 0.011f, 7.f, false},
                        {"motion_mono_th15", &F0, 0.f, 15.f, true}};
  bool retry_seen = false, no_retry_seen = false;
  for (const Case& c : cases) {
    F1.mTcw = pose_z(1.f, c.yaw);  // mVelocity * mLastFrame.mTcw: the true pose, or yawed
    const MotionResult want = motion_expected(F1, *c.last, c.th, c.mono);
    const MotionResult got = g_dry ? want : motion_adapter(F1, *c.last, c.th, c.mono);
    if (got.nmatches != want.nmatches || got.retried != want.retried)
      fail(std::string(c.name) + ": nmatches " + std::to_string(got.nmatches) + " vs " + std::to_string(want.nmatches));
    same_pointers(got.mps, want.mps, c.name);
    (got.retried ? retry_seen : no_retry_seen) = true;
    js += (js.empty() ? "" : ", ") + fmt_motion(c.name, got);
  }
  if (!retry_seen || !no_retry_seen) fail("the motion-model cases must take the 2*th retry once and skip it once");
  F1.mTcw = pose_z(1.f);
  if (g_dry)
    F1.mvpMapPoints = motion_expected(F1, F0, 7.f, false).mps;
  else
    motion_adapter(F1, F0, 7.f, false);  // CurrentFrame's MapPoints from the motion model

  // ---- SearchLocalPoints: local map = KeyFrame 0's and KeyFrame 2's MapPoints ------------------
  KeyFrame K2(F2, nullptr, nullptr);
  add_stereo_mappoints(F2, &K2, pool, 2);
  std::vector<MapPoint*> local;
  for (KeyFrame* k : {&K0, &K2})
    for (MapPoint* p : k->GetMapPointMatches())
      if (p) local.push_back(p);
  {
    std::set<MapPoint*> in_frame(F1.mvpMapPoints.begin(), F1.mvpMapPoints.end());
    std::vector<uint8_t> fl(local.size(), 0);
    for (size_t i = 0; i < local.size(); i++) {
      if (in_frame.count(local[i])) {  // Tracking.cc:1176-1187: already matched, not searched again
        local[i]->mbTrackInView = false;
        fl[i] = ORBFE_MPF_SEEN;
      } else if (local[i]->isBad()) {
        fl[i] = ORBFE_MPF_BAD;
      }
    }
    Geometry g(local, fl);
    View fv;
    frame_view(F1, fv);
    const size_t m = local.size();
    std::vector<uint8_t> of(m);
    std::vector<float> px(m), py(m), pxr(m), vc(m);
    std::vector<int32_t> lvl(m);
    orbfe_frustum_out out{of.data(), px.data(), py.data(), pxr.data(), lvl.data(), vc.data()};
    int nin = 0;
    orbref_is_in_frustum(&fv.v, &g.v, F1.mTcw.ptr<float>(), F1.mfLogScaleFactor, 0.5f, &out, &nin);
    for (size_t i = 0; i < m; i++) {  // Frame::isInFrustum's writes (Frame.cc:365-371)
      if (fl[i]) continue;
      MapPoint* p = local[i];
      p->mbTrackInView = (of[i] & ORBFE_MPF_TRACK_IN_VIEW) != 0;
      if (!p->mbTrackInView) continue;
      p->mTrackProjX = px[i];
      p->mTrackProjY = py[i];
      p->mTrackProjXR = pxr[i];
      p->mnTrackScaleLevel = lvl[i];
      p->mTrackViewCos = vc[i];
    }
    const std::vector<MapPoint*> before = F1.mvpMapPoints;
    for (float th : {5.f, 1.f}) {  // th 1 last: it is the state the next steps start from
      F1.mvpMapPoints = before;
      // expected: the local view packed here, the oracle, the reference's assignment loop
      std::vector<uint8_t> lf(m, 0), ld(m * 32, 0);
      for (size_t i = 0; i < m; i++) {
        MapPoint* p = local[i];
        lf[i] = (p->mbTrackInView ? ORBFE_MPF_TRACK_IN_VIEW : 0u) | (p->isBad() ? ORBFE_MPF_BAD : 0u) |
                (p->Observations() > 0 ? ORBFE_MPF_OBSERVED : 0u);
        const cv::Mat d = p->GetDescriptor();
        std::memcpy(&ld[i * 32], d.data, 32);
        px[i] = p->mTrackProjX;
        py[i] = p->mTrackProjY;
        pxr[i] = p->mTrackProjXR;
        lvl[i] = p->mnTrackScaleLevel;
        vc[i] = p->mTrackViewCos;
      }
      orbfe_local_mappoints lm{(int32_t)m, lf.data(), px.data(), py.data(), pxr.data(), lvl.data(), vc.data(),
                               ld.data()};
      View cur;
      frame_view(F1, cur);
      std::vector<int32_t> best(m, -1);
      int nwant = 0;
      orbref_search_by_projection_local(&cur.v, &lm, th, 0.8f, best.data(), &nwant);
      std::vector<MapPoint*> want = before;
      apply_local(best, want, local);
      ORBmatcher matcher(0.8);  // Tracking.cc:1205
      if (g_dry) F1.mvpMapPoints = want;
      const int ngot = g_dry ? nwant : matcher.SearchByProjection(F1, local, th);
      const std::string tag = "local_th" + std::to_string((int)th);
      if (ngot != nwant) fail(tag + ": nmatches " + std::to_string(ngot) + " vs " + std::to_string(nwant));
      same_pointers(F1.mvpMapPoints, want, tag);
      char b[160];
      std::snprintf(b, sizeof b, ", \"%s\": {\"in_view\": %d, \"nmatches\": %d, \"assigned\": %d}", tag.c_str(), nin,
                    ngot, count_set(F1.mvpMapPoints));
      js += b;
    }
  }

  // ---- LocalMapping::CreateNewMapPoints: SearchForTriangulation(KF1, KF0 / KF2) -----------------
  KeyFrame K1(F1, nullptr, nullptr);
  for (auto kb : {std::make_pair(&K0, "kf0"), std::make_pair(&K2, "kf2")}) {  // pKF2: the previous and the next KeyFrame
    KeyFrame* KB = kb.first;
    const char* name = kb.second;
    // ComputeF12 (LocalMapping.cc:684-700) in double, stored as the CV_32F matrix the reference passes
    const cv::Mat T1 = K1.GetPose(), T2 = KB->GetPose();
    double R1[9], t1[3], R2[9], t2[3], R12[9], t12[3];
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) {
        R1[i * 3 + j] = T1.at<float>(i, j);
        R2[i * 3 + j] = T2.at<float>(i, j);
      }
      t1[i] = T1.at<float>(i, 3);
      t2[i] = T2.at<float>(i, 3);
    }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += R1[i * 3 + k] * R2[j * 3 + k];
        R12[i * 3 + j] = s;
      }
    for (int i = 0; i < 3; i++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += R12[i * 3 + k] * t2[k];
      t12[i] = -s + t1[i];
    }
    const double tx[9] = {0, -t12[2], t12[1], t12[2], 0, -t12[0], -t12[1], t12[0], 0};
    double E[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += tx[i * 3 + k] * R12[k * 3 + j];
        E[i * 3 + j] = s;
      }
    const double f = kFx, cx = kCx, cy = kCy;  // K^-1 = [1/f 0 -cx/f; 0 1/f -cy/f; 0 0 1]
    const double Ki[9] = {1 / f, 0, -cx / f, 0, 1 / f, -cy / f, 0, 0, 1};
    double KtE[9], F12d[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += Ki[k * 3 + i] * E[k * 3 + j];
        KtE[i * 3 + j] = s;
      }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += KtE[i * 3 + k] * Ki[k * 3 + j];
        F12d[i * 3 + j] = s;
      }
    cv::Mat F12(3, 3, CV_32F);
    for (int i = 0; i < 9; i++) F12.ptr<float>()[i] = (float)F12d[i];
    // the epipole of KF1 in KF2 as the adapter computes it (ORBmatcher.cc:678-684)
    const cv::Mat C2 = KB->GetRotation() * K1.GetCameraCenter() + KB->GetTranslation();
    const float invz = 1.0f / C2.at<float>(2);
    const float ex = KB->fx * C2.at<float>(0) * invz + KB->cx, ey = KB->fy * C2.at<float>(1) * invz + KB->cy;
    View v1, v2;
    keyframe_view(&K1, v1);
    keyframe_view(KB, v2);
    Csr fv1(K1.mFeatVec), fv2(KB->mFeatVec);
    for (bool only_stereo : {false, true}) {
      std::vector<int32_t> m12(K1.N, -1);
      int nwant = 0;
      orbref_search_for_triangulation(&v1.v, &v2.v, &fv1.v, &fv2.v, F12.ptr<float>(), ex, ey, only_stereo ? 1 : 0, 0,
                                      m12.data(), &nwant);
      std::vector<std::pair<size_t, size_t>> want;
      for (int i = 0; i < K1.N; i++)  // ORBmatcher.cc:828-836
        if (m12[i] >= 0) want.emplace_back((size_t)i, (size_t)m12[i]);
      ORBmatcher matcher(0.6, false);  // LocalMapping.cc:219
      std::vector<std::pair<size_t, size_t>> got = want;
      const int ngot = g_dry ? nwant : matcher.SearchForTriangulation(&K1, KB, F12, got, only_stereo);
      const std::string tag = std::string("triangulation_") + name + (only_stereo ? "_only_stereo" : "");
      if (ngot != nwant) fail(tag + ": nmatches " + std::to_string(ngot) + " vs " + std::to_string(nwant));
      if (got != want) fail(tag + ": vMatchedPairs differ");
      char b[160];
      std::snprintf(b, sizeof b, ", \"%s\": {\"pairs\": %zu, \"epipole\": [%.3f, %.3f]}", tag.c_str(), got.size(), ex,
                    ey);
      js += b;
    }
  }

  // ---- Tracking::Relocalization on frame 2 against KeyFrame 1 ----------------------------------
  {
    F2.mTcw = pose_z(2.f);
    std::fill(F2.mvpMapPoints.begin(), F2.mvpMapPoints.end(), static_cast<MapPoint*>(nullptr));
    // SearchByBoW(pKF, F, vpMapPointMatches) with ORBmatcher(0.75, true) (Tracking.cc:1451-1466)
    View vk, vf;
    keyframe_view(&K1, vk);
    frame_view(F2, vf);
    Csr fk(K1.mFeatVec), ff(F2.mFeatVec);
    std::vector<int32_t> mf(F2.N, -1);
    int nwant = 0;
    orbref_search_by_bow_kf_frame(&vk.v, &fk.v, &vf.v, &ff.v, 0.75f, 1, mf.data(), &nwant);
    const std::vector<MapPoint*> kmps = K1.GetMapPointMatches();
    std::vector<MapPoint*> want(F2.N, nullptr);
    for (int k = 0; k < F2.N; k++)  // ORBmatcher.cc:283-286 (vpMapPointMatches[realIdxF] = pMP)
      if (mf[k] >= 0) want[k] = kmps[mf[k]];
    ORBmatcher matcher(0.75, true);
    std::vector<MapPoint*> got = want;
    const int ngot = g_dry ? nwant : matcher.SearchByBoW(&K1, F2, got);
    if (ngot != nwant) fail("bow: nmatches " + std::to_string(ngot) + " vs " + std::to_string(nwant));
    same_pointers(got, want, "bow");
    // the PnP stand-in: every other BoW match kept as an inlier (Tracking.cc:1419-1440)
    std::set<MapPoint*> sFound;
    int kept = 0;
    for (int k = 0; k < F2.N; k++)
      if (got[k] && (kept++ % 2 == 0)) {
        F2.mvpMapPoints[k] = got[k];
        sFound.insert(got[k]);
      }
    // SearchByProjection(F, pKF, sFound, 10, 100) with ORBmatcher(0.9, true) (Tracking.cc:1472-1480)
    std::vector<uint8_t> fl(kmps.size(), 0);
    for (size_t i = 0; i < kmps.size(); i++)
      if (MapPoint* p = kmps[i])
        fl[i] = ORBFE_MPF_PRESENT | (p->isBad() ? ORBFE_MPF_BAD : 0u) | (sFound.count(p) ? ORBFE_MPF_SKIP : 0u);
    Geometry g(kmps, fl);
    std::vector<float> ang(K1.N);
    for (int i = 0; i < K1.N; i++) ang[i] = K1.mvKeysUn[i].angle;
    View cur;
    view_common(F2, F2.mvpMapPoints, false, cur);
    cur.v.min_x = Frame::mnMinX;
    cur.v.max_x = Frame::mnMaxX;
    cur.v.min_y = Frame::mnMinY;
    cur.v.max_y = Frame::mnMaxY;
    std::vector<int32_t> best(kmps.size(), -1);
    int nw2 = 0;
    orbref_search_by_projection_keyframe(&cur.v, F2.mTcw.ptr<float>(), &g.v, ang.data(), F2.mfLogScaleFactor, 10.f,
                                         100, 1, best.data(), &nw2);
    std::vector<MapPoint*> want2 = F2.mvpMapPoints;
    apply_with_rotation(best, want2, kmps);
    ORBmatcher matcher2(0.9, true);
    if (g_dry) F2.mvpMapPoints = want2;
    const int ng2 = g_dry ? nw2 : matcher2.SearchByProjection(F2, &K1, sFound, 10, 100);
    if (ng2 != nw2) fail("reloc_projection: nmatches " + std::to_string(ng2) + " vs " + std::to_string(nw2));
    same_pointers(F2.mvpMapPoints, want2, "reloc_projection");
    char b[200];
    std::snprintf(b, sizeof b, ", \"bow\": {\"nmatches\": %d}, \"reloc_projection\": {\"nmatches\": %d, \"assigned\": %d}",
                  ngot, ng2, count_set(F2.mvpMapPoints));
    js += b;
  }

  // ---- LoopClosing::ComputeSim3's SearchByProjection(pKF, Scw, vpPoints, vpMatched, 10) ----------
  {
    // KeyFrame 1 against KeyFrame 2's MapPoints through the identity Sim3 of its own pose
    std::vector<MapPoint*> pts;
    for (MapPoint* p : K2.GetMapPointMatches())
      if (p) pts.push_back(p);
    std::vector<MapPoint*> matched = K1.GetMapPointMatches();  // vpCurrentMatchedPoints
    for (size_t i = 0; i < matched.size(); i++)
      if (i % 3) matched[i] = nullptr;
    const cv::Mat Scw = K1.GetPose();
    View vk;
    keyframe_view(&K1, vk);
    for (int i = 0; i < K1.N; i++) vk.state[i] = matched[i] ? ORBFE_MP_PRESENT : ORBFE_MP_NONE;
    std::set<MapPoint*> already(matched.begin(), matched.end());
    already.erase(nullptr);
    std::vector<uint8_t> fl(pts.size());
    for (size_t i = 0; i < pts.size(); i++)
      fl[i] = ORBFE_MPF_PRESENT | (pts[i]->isBad() ? ORBFE_MPF_BAD : 0u) | (already.count(pts[i]) ? ORBFE_MPF_SKIP : 0u);
    Geometry g(pts, fl);
    std::vector<int32_t> best(pts.size(), -1);
    int nwant = 0;
    orbref_search_by_projection_sim3(&vk.v, Scw.ptr<float>(), &g.v, K1.mfLogScaleFactor, 10, best.data(), &nwant);
    std::vector<MapPoint*> want = matched;
    apply_local(best, want, pts);  // vpMatched[bestIdx] = pMP (ORBmatcher.cc:404-406)
    ORBmatcher matcher(0.75, true);  // LoopClosing.cc:402
    if (g_dry) matched = want;
    const int ngot = g_dry ? nwant : matcher.SearchByProjection(&K1, Scw, pts, matched, 10);
    if (ngot != nwant) fail("sim3_projection: nmatches " + std::to_string(ngot) + " vs " + std::to_string(nwant));
    same_pointers(matched, want, "sim3_projection");
    char b[120];
    std::snprintf(b, sizeof b, ", \"sim3_projection\": {\"nmatches\": %d}", ngot);
    js += b;
  }

  std::printf("MATCHER {%s, \"mappoints\": %zu, \"keypoints\": [%d, %d, %d]}\n", js.c_str(), pool.size(), F0.N, F1.N,
              F2.N);
  std::printf("%s\n", g_fails ? "MISMATCH" : "OK");
  return g_fails ? 1 : 0;
}
