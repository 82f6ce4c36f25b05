// CPU test of the reference-side adapter (adapter/orbfe_pack.hpp, adapter/orbfe_adapter.hpp):
// every ORBmatcher method template instantiated on ORB-SLAM2-shaped test structs (the reference's
// member and method names, its non-const accessors) with a recording matcher in place of the GPU:
// the SoA views it receives are checked field by field against the objects, and canned results
// are applied to the object graph as the reference's loops would (ORBmatcher.cc). No GPU, no
// library: the search itself is covered by the GPU parity tests.
// Exit 0 = all checks passed; prints the first failure otherwise.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <vector>

#include "../../adapter/orbfe_adapter.hpp"

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
      g_fail++;                                                         \
    }                                                                   \
  } while (0)

namespace ref {  // ORB-SLAM2-shaped stand-ins (include/Frame.h, KeyFrame.h, MapPoint.h)

struct Mat {  // a cv::Mat header: shared storage, public `data`
  std::shared_ptr<std::vector<uint8_t>> store;
  uint8_t* data = nullptr;
  static Mat bytes(size_t n, uint8_t seed) {
    Mat m;
    m.store = std::make_shared<std::vector<uint8_t>>(n);
    for (size_t i = 0; i < n; i++) (*m.store)[i] = (uint8_t)(seed * 31 + i * 7);
    m.data = m.store->data();
    return m;
  }
  static Mat floats(std::vector<float> v) {
    Mat m;
    m.store = std::make_shared<std::vector<uint8_t>>(v.size() * 4);
    std::memcpy(m.store->data(), v.data(), v.size() * 4);
    m.data = m.store->data();
    return m;
  }
  const float* f() const { return reinterpret_cast<const float*>(data); }
};

struct KeyPoint {
  struct {
    float x, y;
  } pt;
  float size, angle, response;
  int octave, class_id;
};

struct KeyFrame;
struct MapPoint {
  // public tracking members (MapPoint.h:95-110)
  bool mbTrackInView = false;
  float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0;
  int mnTrackScaleLevel = 0;
  float mTrackViewCos = 0;
  // state behind the reference's (non-const) accessors
  bool bad = false;
  int nobs = 0;
  Mat desc, pos, normal;
  float mfMinDistance = 0, mfMaxDistance = 0;  // protected in the reference; the adapter's friend reads them
  std::map<const KeyFrame*, int> obs;
  MapPoint* replaced_by = nullptr;
  bool isBad() { return bad; }
  int Observations() { return nobs; }
  Mat GetDescriptor() { return desc; }
  Mat GetWorldPos() { return pos; }
  Mat GetNormal() { return normal; }
  bool IsInKeyFrame(KeyFrame* k) { return obs.count(k) > 0; }
  int GetIndexInKeyFrame(KeyFrame* k) { return obs.count(k) ? obs[k] : -1; }
  void AddObservation(KeyFrame* k, size_t idx) {
    obs[k] = (int)idx;
    nobs++;
  }
  void Replace(MapPoint* p) {
    replaced_by = p;
    bad = true;
  }
};

using FeatureVector = std::map<unsigned, std::vector<unsigned>>;  // DBoW2::FeatureVector

struct Frame {
  int N = 0;
  std::vector<KeyPoint> mvKeys, mvKeysUn;
  std::vector<float> mvuRight;
  Mat mDescriptors;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
  int mnScaleLevels = 8;
  std::vector<float> mvScaleFactors, mvLevelSigma2;
  float mfLogScaleFactor = 0.18232156f;
  static float mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv;
  float fx = 718.856f, fy = 718.856f, cx = 607.19f, cy = 185.22f, mbf = 386.1448f, mb = 0.5372f;
  Mat mTcw;
  FeatureVector mFeatVec;
};
float Frame::mnMinX = 0.f, Frame::mnMaxX = 1241.f, Frame::mnMinY = 0.f, Frame::mnMaxY = 376.f;
float Frame::mfGridElementWidthInv = 64.f / 1241.f, Frame::mfGridElementHeightInv = 48.f / 376.f;

struct KeyFrame {
  int N = 0;
  std::vector<KeyPoint> mvKeys, mvKeysUn;
  std::vector<float> mvuRight;
  Mat mDescriptors;
  int mnScaleLevels = 8;
  std::vector<float> mvScaleFactors, mvLevelSigma2;
  float mfLogScaleFactor = 0.18232156f;
  int mnMinX = 0, mnMaxX = 1241, mnMinY = 0, mnMaxY = 376;  // const int in KeyFrame.h:202-205
  float mfGridElementWidthInv = 64.f / 1241.f, mfGridElementHeightInv = 48.f / 376.f;
  float fx = 718.856f, fy = 718.856f, cx = 607.19f, cy = 185.22f, mbf = 386.1448f, mb = 0.5372f;
  FeatureVector mFeatVec;
  std::vector<MapPoint*> mps;
  Mat pose, center;
  std::vector<MapPoint*> GetMapPointMatches() { return mps; }
  std::set<MapPoint*> GetMapPoints() {
    std::set<MapPoint*> s;
    for (MapPoint* p : mps)
      if (p && !p->isBad()) s.insert(p);
    return s;
  }
  MapPoint* GetMapPoint(size_t i) { return mps[i]; }
  void AddMapPoint(MapPoint* p, size_t i) { mps[i] = p; }
  Mat GetPose() { return pose; }
  Mat GetCameraCenter() { return center; }
};

struct Point2f {
  float x, y;
};

}  // namespace ref

// ---- the recording matcher (orbfe::Matcher's signatures) ---------------------------------------
struct Recorder {
  orbfe_frame_view f1{}, f2{};
  std::vector<orbfe_keypoint> k1, k2;
  std::vector<uint8_t> s1, s2;
  orbfe_local_mappoints local{};
  orbfe_lastframe_mappoints last{};
  std::vector<uint8_t> flags, flags2, desc;     // copies: the packers free their arrays after the call
  std::vector<float> pos, angle, dmin, px, py, pxr, vcos;
  std::vector<int32_t> level, octave;
  orbfe_feature_vector fv1{}, fv2{};
  std::vector<uint32_t> ids1;
  std::vector<int32_t> off1, idx1;
  std::vector<float> tcw;
  float th = 0, lsf = 0;
  bool mono = false;
  int orbdist = 0;
  std::vector<int32_t> result;  // returned as best / match vector
  int ret = 0;

  void keep_frame(const orbfe_frame_view& v, orbfe_frame_view& o, std::vector<orbfe_keypoint>& k,
                  std::vector<uint8_t>& s) {
    o = v;
    k.assign(v.keys_un, v.keys_un + v.n);
    s.assign(v.mp_state, v.mp_state + v.n);
  }
  void keep_fv(const orbfe_feature_vector& f) {
    ids1.assign(f.node_ids, f.node_ids + f.n_nodes);
    off1.assign(f.offsets, f.offsets + f.n_nodes + 1);
    idx1.assign(f.indices, f.indices + off1.back());
  }
  int SearchByProjection(const orbfe_frame_view& F, const orbfe_local_mappoints& mps, float t,
                         std::vector<int32_t>& best) {
    keep_frame(F, f1, k1, s1);
    local = mps;
    flags.assign(mps.flags, mps.flags + mps.m);
    px.assign(mps.proj_x, mps.proj_x + mps.m);
    py.assign(mps.proj_y, mps.proj_y + mps.m);
    pxr.assign(mps.proj_xr, mps.proj_xr + mps.m);
    vcos.assign(mps.view_cos, mps.view_cos + mps.m);
    level.assign(mps.level, mps.level + mps.m);
    desc.assign(mps.descriptors, mps.descriptors + 32 * mps.m);
    th = t;
    best = result;
    return ret;
  }
  int SearchByProjection(const orbfe_frame_view& cur, const orbfe_lastframe_mappoints& l, const float* t_cur,
                         float t, bool m, std::vector<int32_t>& best) {
    keep_frame(cur, f1, k1, s1);
    last = l;
    flags.assign(l.flags, l.flags + l.n);
    pos.assign(l.world_pos, l.world_pos + 3 * l.n);
    angle.assign(l.angle, l.angle + l.n);
    octave.assign(l.octave, l.octave + l.n);
    desc.assign(l.descriptors, l.descriptors + 32 * l.n);
    tcw.assign(t_cur, t_cur + 12);
    th = t;
    mono = m;
    best = result;
    return ret;
  }
  int SearchForTriangulation(const orbfe_frame_view& a, const orbfe_frame_view& b, const orbfe_feature_vector& fa,
                             const orbfe_feature_vector& fb, const float* f12, float ex, float ey,
                             std::vector<std::pair<size_t, size_t>>& pairs, bool only_stereo) {
    keep_frame(a, f1, k1, s1);
    keep_frame(b, f2, k2, s2);
    keep_fv(fa);
    fv2 = fb;
    tcw.assign(f12, f12 + 9);
    tcw.push_back(ex);
    tcw.push_back(ey);
    mono = only_stereo;
    pairs.clear();
    for (size_t i = 0; i < result.size(); i++)
      if (result[i] >= 0) pairs.emplace_back(i, (size_t)result[i]);
    return ret;
  }
  int SearchByBoW(const orbfe_frame_view& kf, const orbfe_feature_vector& kfv, const orbfe_frame_view& F,
                  const orbfe_feature_vector& ffv, std::vector<int32_t>& m) {
    keep_frame(kf, f1, k1, s1);
    keep_frame(F, f2, k2, s2);
    keep_fv(kfv);
    fv2 = ffv;
    m = result;
    return ret;
  }
  int SearchByBoW12(const orbfe_frame_view& a, const orbfe_feature_vector& fa, const orbfe_frame_view& b,
                    const orbfe_feature_vector& fb, std::vector<int32_t>& m) {
    return SearchByBoW(a, fa, b, fb, m);
  }
  void keep_geo(const orbfe_mappoint_geometry& g, std::vector<uint8_t>& fl) {
    fl.assign(g.flags, g.flags + g.m);
    pos.assign(g.world_pos, g.world_pos + 3 * g.m);
    dmin.assign(g.min_distance, g.min_distance + g.m);
  }
  int SearchByProjection(const orbfe_frame_view& cur, const float* t_cur, const orbfe_mappoint_geometry& g,
                         const float* ang, float l, float t, int od, std::vector<int32_t>& best) {
    keep_frame(cur, f1, k1, s1);
    keep_geo(g, flags);
    angle.assign(ang, ang + g.m);
    tcw.assign(t_cur, t_cur + 12);
    lsf = l;
    th = t;
    orbdist = od;
    best = result;
    return ret;
  }
  int SearchByProjectionSim3(const orbfe_frame_view& kf, const float* scw, const orbfe_mappoint_geometry& g, float l,
                             int t, std::vector<int32_t>& best) {
    keep_frame(kf, f1, k1, s1);
    keep_geo(g, flags);
    tcw.assign(scw, scw + 12);
    lsf = l;
    th = (float)t;
    best = result;
    return ret;
  }
  int Fuse(const orbfe_frame_view& kf, const float* t, const float* ow, const orbfe_mappoint_geometry& g, float l,
           float thr, std::vector<int32_t>& best) {
    keep_frame(kf, f1, k1, s1);
    keep_geo(g, flags);
    tcw.assign(t, t + 12);
    tcw.insert(tcw.end(), ow, ow + 3);
    lsf = l;
    th = thr;
    best = result;
    return ret;
  }
  int FuseSim3(const orbfe_frame_view& kf, const float* scw, const orbfe_mappoint_geometry& g, float l, float thr,
               std::vector<int32_t>& best) {
    keep_frame(kf, f1, k1, s1);
    keep_geo(g, flags);
    tcw.assign(scw, scw + 12);
    lsf = l;
    th = thr;
    best = result;
    return ret;
  }
  int SearchBySim3(const orbfe_frame_view& a, const orbfe_frame_view& b, const orbfe_mappoint_geometry& g1,
                   const orbfe_mappoint_geometry& g2, const float* t1w, const float* t2w, float s12, const float* r12,
                   const float* t12, float l1, float l2, float thr, std::vector<int32_t>& m12) {
    keep_frame(a, f1, k1, s1);
    keep_frame(b, f2, k2, s2);
    keep_geo(g1, flags);
    flags2.assign(g2.flags, g2.flags + g2.m);
    tcw.assign(t1w, t1w + 12);
    tcw.insert(tcw.end(), t2w, t2w + 12);
    tcw.push_back(s12);
    tcw.insert(tcw.end(), r12, r12 + 9);
    tcw.insert(tcw.end(), t12, t12 + 3);
    lsf = l1 + 100 * l2;
    th = thr;
    m12 = result;
    return ret;
  }
  int SearchForInitialization(const orbfe_frame_view& a, const orbfe_frame_view& b, std::vector<float>& prev,
                              std::vector<int32_t>& m12, int window) {
    keep_frame(a, f1, k1, s1);
    keep_frame(b, f2, k2, s2);
    pos = prev;
    for (float& v : prev) v += 1.0f;  // the library updates vbPrevMatched in place
    orbdist = window;
    m12 = result;
    return ret;
  }
};

// ---- scene builders ---------------------------------------------------------------------------
static std::vector<ref::KeyPoint> keypoints(int n, float off) {
  std::vector<ref::KeyPoint> k(n);
  for (int i = 0; i < n; i++)
    k[i] = ref::KeyPoint{{off + 10.f * i, off + 3.f * i}, 31.f * (1 + i % 3), 1.5f * i, (float)(20 + i), i % 8, -1};
  return k;
}

static ref::MapPoint* new_mp(std::vector<std::unique_ptr<ref::MapPoint>>& pool, int seed, int nobs, bool bad) {
  pool.emplace_back(new ref::MapPoint());
  ref::MapPoint* p = pool.back().get();
  p->desc = ref::Mat::bytes(32, (uint8_t)seed);
  p->pos = ref::Mat::floats({1.f * seed, 2.f * seed, 3.f + seed});
  p->normal = ref::Mat::floats({0.f, 0.f, 1.f});
  p->mfMinDistance = 0.5f + seed;
  p->mfMaxDistance = 9.f + seed;
  p->nobs = nobs;
  p->bad = bad;
  p->mbTrackInView = seed % 4 != 1;
  p->mTrackProjX = 100.f + seed;
  p->mTrackProjY = 50.f + seed;
  p->mTrackProjXR = 90.f + seed;
  p->mnTrackScaleLevel = seed % 8;
  p->mTrackViewCos = 0.9f;
  return p;
}

static void fill_frame(ref::Frame& f, int n, float off) {
  f.N = n;
  f.mvKeys = keypoints(n, off + 0.25f);  // distorted keypoints differ from the undistorted ones
  f.mvKeysUn = keypoints(n, off);
  f.mvuRight.resize(n);
  for (int i = 0; i < n; i++) f.mvuRight[i] = i % 2 ? -1.f : off + 10.f * i - 5.f;
  f.mDescriptors = ref::Mat::bytes((size_t)n * 32, 9);
  f.mvpMapPoints.assign(n, nullptr);
  f.mvbOutlier.assign(n, false);
  f.mvScaleFactors = {1.f, 1.2f, 1.44f, 1.728f, 2.0736f, 2.48832f, 2.985984f, 3.5831808f};
  f.mvLevelSigma2 = {1.f, 1.44f, 2.0736f, 2.985984f, 4.2998f, 6.1917f, 8.9161f, 12.8392f};
  std::vector<float> T(16, 0.f);
  for (int i = 0; i < 16; i++) T[i] = 0.5f * i + off;
  f.mTcw = ref::Mat::floats(T);
}

static std::vector<uint8_t> states(const ref::Frame& f) {  // the keypoints' MapPoint state before a call
  std::vector<uint8_t> s(f.N);
  for (int i = 0; i < f.N; i++) {
    const ref::MapPoint* p = f.mvpMapPoints[i];
    s[i] = !p ? ORBFE_MP_NONE : p->nobs > 0 ? ORBFE_MP_OBSERVED : ORBFE_MP_PRESENT;
  }
  return s;
}

static void check_frame_view(const orbfe_frame_view& v, const std::vector<orbfe_keypoint>& k,
                             const std::vector<uint8_t>& s, const ref::Frame& f, const std::vector<uint8_t>& st0) {
  CHECK(v.n == f.N && (int)k.size() == f.N);
  for (int i = 0; i < f.N; i++) {
    const ref::KeyPoint& r = f.mvKeysUn[i];
    CHECK(k[i].x == r.pt.x && k[i].y == r.pt.y && k[i].size == r.size && k[i].angle == r.angle &&
          k[i].response == r.response && k[i].octave == r.octave && k[i].class_id == r.class_id);
  }
  CHECK(s == st0);
  CHECK(v.u_right == f.mvuRight.data() && v.descriptors == f.mDescriptors.data);
  CHECK(v.nlevels == f.mnScaleLevels && v.scale_factors == f.mvScaleFactors.data() &&
        v.level_sigma2 == f.mvLevelSigma2.data());
  CHECK(v.min_x == ref::Frame::mnMinX && v.max_x == ref::Frame::mnMaxX && v.min_y == ref::Frame::mnMinY &&
        v.max_y == ref::Frame::mnMaxY);
  CHECK(v.grid_inv_w == ref::Frame::mfGridElementWidthInv && v.grid_inv_h == ref::Frame::mfGridElementHeightInv);
  CHECK(v.fx == f.fx && v.fy == f.fy && v.cx == f.cx && v.cy == f.cy && v.bf == f.mbf && v.b == f.mb);
  CHECK(v.grid_origin_set == 0);
}

static auto dist_of = [](ref::MapPoint* p, float& a, float& b) {
  a = p->mfMinDistance;
  b = p->mfMaxDistance;
};

int main() {
  using namespace orbfe_adapter;
  std::vector<std::unique_ptr<ref::MapPoint>> pool;

  // ---- SearchByProjection(F, vpMapPoints, th): LocalMapPack + ascending application ----------
  {
    ref::Frame F;
    fill_frame(F, 12, 5.f);
    F.mvpMapPoints[3] = new_mp(pool, 40, 2, false);  // OBSERVED
    F.mvpMapPoints[5] = new_mp(pool, 41, 0, false);  // PRESENT
    std::vector<ref::MapPoint*> vp;
    for (int i = 0; i < 8; i++) vp.push_back(new_mp(pool, i, i % 3, i == 6));
    Recorder m;
    m.result = {4, -1, 7, 4, -1, -1, -1, 9};  // MapPoint 3 takes keypoint 4 after MapPoint 0
    m.ret = 3;
    const std::vector<uint8_t> st0 = states(F);
    const int n = search_by_projection_local(m, F, vp, 1.0f);
    CHECK(n == 3 && m.th == 1.0f);
    check_frame_view(m.f1, m.k1, m.s1, F, st0);
    CHECK(m.s1[3] == ORBFE_MP_OBSERVED && m.s1[5] == ORBFE_MP_PRESENT && m.s1[0] == ORBFE_MP_NONE);
    CHECK(m.local.m == 8);
    for (int i = 0; i < 8; i++) {
      ref::MapPoint* p = vp[i];
      const unsigned want = (p->mbTrackInView ? ORBFE_MPF_TRACK_IN_VIEW : 0u) | (p->bad ? ORBFE_MPF_BAD : 0u) |
                            (p->nobs > 0 ? ORBFE_MPF_OBSERVED : 0u);
      CHECK(m.flags[i] == want);
      if (p->mbTrackInView && !p->bad) {
        CHECK(m.px[i] == p->mTrackProjX && m.py[i] == p->mTrackProjY && m.pxr[i] == p->mTrackProjXR &&
              m.level[i] == p->mnTrackScaleLevel && m.vcos[i] == p->mTrackViewCos);
        CHECK(std::memcmp(&m.desc[32 * i], p->desc.data, 32) == 0);
      }
    }
    CHECK(F.mvpMapPoints[4] == vp[3] && F.mvpMapPoints[7] == vp[2] && F.mvpMapPoints[9] == vp[7]);
    CHECK(F.mvpMapPoints[3] != nullptr && F.mvpMapPoints[0] == nullptr);
  }

  // ---- SearchByProjection(CurrentFrame, LastFrame, th, bMono): LastFramePack + undo codes -----
  {
    ref::Frame C, Lf;
    fill_frame(C, 10, 3.f);
    fill_frame(Lf, 7, 8.f);
    for (int i = 0; i < 7; i++)
      if (i != 2) Lf.mvpMapPoints[i] = new_mp(pool, 60 + i, i % 2, false);
    Lf.mvbOutlier[4] = true;
    Recorder m;
    // A..G = last-frame MapPoints 0..6: 0 -> kp 2; 1 none; 3 -> kp 4 then undone; 4 (outlier)
    // none; 5 -> kp 4 again (kept, but kp 4 is NULLed by 3's undo, as in the reference);
    // 6 -> kp 2 then undone (kp 2 ends NULL although 0 assigned it first)
    m.result = {2, -1, -1, -2 - 4, -1, 4, -2 - 2};
    m.ret = 1;
    const std::vector<uint8_t> st0 = states(C);
    const int n = search_by_projection_lastframe(m, C, Lf, 7.f, false);
    CHECK(n == 1 && m.th == 7.f && !m.mono);
    check_frame_view(m.f1, m.k1, m.s1, C, st0);
    CHECK(m.last.n == 7);
    for (int i = 0; i < 7; i++) {
      ref::MapPoint* p = Lf.mvpMapPoints[i];
      const unsigned want = !p ? 0u
                               : ORBFE_MPF_PRESENT | (Lf.mvbOutlier[i] ? ORBFE_MPF_OUTLIER : 0u) |
                                     (p->nobs > 0 ? ORBFE_MPF_OBSERVED : 0u);
      CHECK(m.flags[i] == want);
      CHECK(m.octave[i] == Lf.mvKeys[i].octave && m.angle[i] == Lf.mvKeysUn[i].angle);
      if (p && !Lf.mvbOutlier[i]) {
        CHECK(m.pos[3 * i] == p->pos.f()[0] && m.pos[3 * i + 1] == p->pos.f()[1] && m.pos[3 * i + 2] == p->pos.f()[2]);
        CHECK(std::memcmp(&m.desc[32 * i], p->desc.data, 32) == 0);
      }
    }
    for (int k = 0; k < 12; k++) CHECK(m.last.tcw_last[k] == Lf.mTcw.f()[k] && m.tcw[k] == C.mTcw.f()[k]);
    CHECK(C.mvpMapPoints[2] == nullptr && C.mvpMapPoints[4] == nullptr);
    for (int k = 0; k < 10; k++) CHECK(C.mvpMapPoints[k] == nullptr);
    // a plain assignment survives
    ref::Frame C2;
    fill_frame(C2, 10, 3.f);
    m.result = {2, -1, -1, -2 - 4, -1, 6, -1};
    search_by_projection_lastframe(m, C2, Lf, 15.f, true);
    CHECK(m.mono && m.th == 15.f);
    CHECK(C2.mvpMapPoints[2] == Lf.mvpMapPoints[0] && C2.mvpMapPoints[6] == Lf.mvpMapPoints[5] &&
          C2.mvpMapPoints[4] == nullptr);
  }

  // ---- SearchForTriangulation: KeyFrame views + FeatureVector CSR ------------------------------
  {
    ref::KeyFrame K1, K2;
    for (ref::KeyFrame* k : {&K1, &K2}) {
      k->N = 6;
      k->mvKeysUn = keypoints(6, 2.f);
      k->mvuRight.assign(6, -1.f);
      k->mDescriptors = ref::Mat::bytes(6 * 32, 3);
      k->mvScaleFactors.assign(8, 1.f);
      k->mvLevelSigma2.assign(8, 1.f);
      k->mps.assign(6, nullptr);
    }
    K1.mps[1] = new_mp(pool, 80, 1, false);
    K1.mFeatVec = {{12u, {0u, 3u}}, {7u, {1u}}, {40u, {2u, 4u, 5u}}};
    K2.mFeatVec = {{7u, {0u, 1u}}};
    Recorder m;
    m.result = {3, -1, 0, -1, 5, -1};
    m.ret = 3;
    std::vector<std::pair<size_t, size_t>> pairs;
    const float F12[9] = {1, 2, 3, 4, 5, 6, 7, 8, 9};
    const int n = search_for_triangulation(m, &K1, &K2, F12, 600.f, 180.f, pairs, false);
    CHECK(n == 3 && pairs.size() == 3 && pairs[0] == std::make_pair((size_t)0, (size_t)3) && pairs[2].first == 4);
    CHECK(m.ids1 == (std::vector<uint32_t>{7u, 12u, 40u}));
    CHECK(m.off1 == (std::vector<int32_t>{0, 1, 3, 6}));
    CHECK(m.idx1 == (std::vector<int32_t>{1, 0, 3, 2, 4, 5}));
    CHECK(m.fv2.n_nodes == 1);
    CHECK(m.s1[1] == ORBFE_MP_OBSERVED && m.f1.min_x == 0.f && m.f1.max_x == 1241.f && m.f1.n == 6);
    CHECK(m.tcw[8] == 9.f && m.tcw[9] == 600.f && m.tcw[10] == 180.f);
  }

  // ---- SearchByBoW(KF, F) and (KF1, KF2): KeyFrame packing (BAD, grid origin) + mapping --------
  {
    ref::KeyFrame K;
    K.N = 5;
    K.mvKeysUn = keypoints(5, 1.f);
    K.mvuRight.assign(5, -1.f);
    K.mDescriptors = ref::Mat::bytes(5 * 32, 4);
    K.mvScaleFactors.assign(8, 1.f);
    K.mvLevelSigma2.assign(8, 1.f);
    K.mps = {new_mp(pool, 90, 2, false), nullptr, new_mp(pool, 91, 0, true), new_mp(pool, 92, 0, false), nullptr};
    ref::Frame F;
    fill_frame(F, 6, 0.f);
    Recorder m;
    m.result = {-1, 0, 3, -1, 2, -1};
    m.ret = 3;
    std::vector<ref::MapPoint*> out;
    const int n = search_by_bow(m, &K, F, out, 0.5f, 0.25f);
    CHECK(n == 3 && out.size() == 6);
    CHECK(out[1] == K.mps[0] && out[2] == K.mps[3] && out[4] == K.mps[2] && out[0] == nullptr);
    CHECK(m.s1[0] == ORBFE_MP_OBSERVED && m.s1[1] == ORBFE_MP_NONE && m.s1[2] == ORBFE_MP_BAD &&
          m.s1[3] == ORBFE_MP_PRESENT);
    CHECK(m.f1.grid_origin_set == 1 && m.f1.grid_min_x == 0.5f && m.f1.grid_min_y == 0.25f);
    ref::KeyFrame K2 = K;
    m.result = {4, -1, -1, 0, -1};
    std::vector<ref::MapPoint*> m12;
    search_by_bow12(m, &K, &K2, m12, 0.f, 0.f);
    CHECK(m12.size() == 5 && m12[0] == nullptr && m12[3] == K2.mps[0]);
  }

  // ---- SearchByProjection(F, KF, sAlreadyFound, th, ORBdist): GeometryPack flags, undo codes ---
  {
    ref::KeyFrame K;
    K.N = 5;
    K.mvKeysUn = keypoints(5, 4.f);
    K.mps = {new_mp(pool, 100, 1, false), new_mp(pool, 101, 1, true), nullptr, new_mp(pool, 103, 1, false),
             new_mp(pool, 104, 1, false)};
    std::set<ref::MapPoint*> found = {K.mps[3]};
    ref::Frame C;
    fill_frame(C, 8, 1.f);
    Recorder m;
    m.result = {6, -1, -1, -1, -2 - 1};
    m.ret = 1;
    search_by_projection_keyframe(m, C, &K, found, 10.f, 100, dist_of);
    CHECK(m.flags[0] == ORBFE_MPF_PRESENT && m.flags[1] == (ORBFE_MPF_PRESENT | ORBFE_MPF_BAD) && m.flags[2] == 0 &&
          m.flags[3] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP) && m.flags[4] == ORBFE_MPF_PRESENT);
    CHECK(m.dmin[0] == K.mps[0]->mfMinDistance && m.pos[3 * 4 + 2] == K.mps[4]->pos.f()[2]);
    for (int i = 0; i < 5; i++) CHECK(m.angle[i] == K.mvKeysUn[i].angle);
    CHECK(m.orbdist == 100 && m.lsf == C.mfLogScaleFactor && m.tcw[11] == C.mTcw.f()[11]);
    CHECK(C.mvpMapPoints[6] == K.mps[0] && C.mvpMapPoints[1] == nullptr);
  }

  // ---- SearchByProjection(KF, Scw, vpPoints, vpMatched, th) --------------------------------------
  {
    ref::KeyFrame K;
    K.N = 4;
    K.mvKeysUn = keypoints(4, 0.f);
    K.mps.assign(4, nullptr);
    std::vector<ref::MapPoint*> pts = {new_mp(pool, 110, 1, false), new_mp(pool, 111, 1, false),
                                       new_mp(pool, 112, 1, true)};
    std::vector<ref::MapPoint*> matched = {nullptr, pts[1], nullptr, nullptr};
    Recorder m;
    m.result = {2, -1, -1};
    m.ret = 1;
    const float S[16] = {2, 0, 0, 1, 0, 2, 0, 2, 0, 0, 2, 3, 0, 0, 0, 1};
    search_by_projection_sim3(m, &K, S, pts, matched, 10, dist_of, 0.f, 0.f);
    CHECK(m.s1[1] == ORBFE_MP_PRESENT && m.s1[0] == ORBFE_MP_NONE);
    CHECK(m.flags[0] == ORBFE_MPF_PRESENT && m.flags[1] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP) &&
          m.flags[2] == (ORBFE_MPF_PRESENT | ORBFE_MPF_BAD));
    CHECK(m.tcw[3] == 1.f && m.tcw[11] == 3.f && m.th == 10.f);
    CHECK(matched[2] == pts[0] && matched[1] == pts[1]);
  }

  // ---- Fuse(KF, vpMapPoints, th): replace / add in order, re-tested at application --------------
  {
    ref::KeyFrame K;
    K.N = 6;
    K.mvKeysUn = keypoints(6, 0.f);
    K.pose = ref::Mat::floats(std::vector<float>(16, 1.f));
    K.center = ref::Mat::floats({7.f, 8.f, 9.f});
    ref::MapPoint* strong = new_mp(pool, 120, 5, false);  // in the KF at kp 1, more observations
    ref::MapPoint* weak = new_mp(pool, 121, 1, false);    // in the KF at kp 2, fewer observations
    K.mps = {nullptr, strong, weak, nullptr, nullptr, nullptr};
    ref::MapPoint* a = new_mp(pool, 122, 2, false);  // -> kp 1: a replaced by strong
    ref::MapPoint* b = new_mp(pool, 123, 2, false);  // -> kp 2: weak replaced by b
    ref::MapPoint* c = new_mp(pool, 124, 2, false);  // -> kp 3: added
    ref::MapPoint* d = new_mp(pool, 125, 2, false);  // -> kp 3 as well: now occupied by c -> replace
    ref::MapPoint* e = new_mp(pool, 126, 2, false);  // in the KF already: SKIP, never applied
    e->obs[&K] = 5;
    std::vector<ref::MapPoint*> vp = {a, b, c, d, e, nullptr};
    Recorder m;
    m.result = {1, 2, 3, 3, -1, -1};
    const int nf = fuse(m, &K, vp, 3.f, dist_of, 0.f, 0.f);
    CHECK(m.flags[4] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP) && m.flags[5] == 0 && m.flags[0] == ORBFE_MPF_PRESENT);
    CHECK(m.tcw[12] == 7.f && m.tcw[14] == 9.f);
    CHECK(a->replaced_by == strong && weak->replaced_by == b);
    CHECK(K.mps[3] == c && c->obs.count(&K) && c->obs[&K] == 3);
    CHECK(nf == 4);
  }

  // ---- Fuse(KF, Scw, vpPoints, th, vpReplacePoint) ----------------------------------------------
  {
    ref::KeyFrame K;
    K.N = 4;
    K.mvKeysUn = keypoints(4, 0.f);
    ref::MapPoint* in = new_mp(pool, 130, 3, false);
    K.mps = {in, nullptr, nullptr, nullptr};
    std::vector<ref::MapPoint*> pts = {new_mp(pool, 131, 1, false), new_mp(pool, 132, 1, false), in};
    std::vector<ref::MapPoint*> repl(3, nullptr);
    Recorder m;
    m.result = {0, 2, -1};
    m.ret = 2;
    const float S[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const int nf = fuse_sim3(m, &K, S, pts, 4.f, repl, dist_of, 0.f, 0.f);
    CHECK(nf == 2 && m.flags[2] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP));
    CHECK(repl[0] == in && repl[1] == nullptr && K.mps[2] == pts[1] && pts[1]->obs[&K] == 2);
  }

  // ---- SearchBySim3: vbAlreadyMatched from vpMatches12 and GetIndexInKeyFrame ------------------
  {
    ref::KeyFrame K1, K2;
    for (ref::KeyFrame* k : {&K1, &K2}) {
      k->N = 4;
      k->mvKeysUn = keypoints(4, 0.f);
      k->pose = ref::Mat::floats(std::vector<float>(16, 2.f));
    }
    K1.mps = {new_mp(pool, 140, 1, false), new_mp(pool, 141, 1, false), nullptr, new_mp(pool, 143, 1, true)};
    K2.mps = {new_mp(pool, 150, 1, false), nullptr, new_mp(pool, 152, 1, false), new_mp(pool, 153, 1, false)};
    K2.mps[2]->obs[&K2] = 2;
    std::vector<ref::MapPoint*> v12 = {nullptr, K2.mps[2], nullptr, nullptr};  // kp 1 matched to KF2 kp 2
    Recorder m;
    m.result = {3, -1, -1, -1};
    m.ret = 1;
    const float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0.1f, 0.2f, 0.3f};
    search_by_sim3(m, &K1, &K2, v12, 1.5f, R, t, 7.5f, dist_of, 0.f, 0.f);
    CHECK(m.flags[1] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP) && m.flags[0] == ORBFE_MPF_PRESENT && m.flags[2] == 0 &&
          m.flags[3] == (ORBFE_MPF_PRESENT | ORBFE_MPF_BAD));
    CHECK(m.flags2[2] == (ORBFE_MPF_PRESENT | ORBFE_MPF_SKIP) && m.flags2[0] == ORBFE_MPF_PRESENT);
    CHECK(m.tcw[24] == 1.5f && m.tcw[25] == 1.f && m.tcw[36] == 0.3f);
    CHECK(v12[0] == K2.mps[3] && v12[1] == K2.mps[2]);
  }

  // ---- SearchForInitialization: vbPrevMatched updated in place -----------------------------------
  {
    ref::Frame F1, F2;
    fill_frame(F1, 3, 0.f);
    fill_frame(F2, 4, 1.f);
    std::vector<ref::Point2f> prev = {{1.f, 2.f}, {3.f, 4.f}, {5.f, 6.f}};
    std::vector<int> m12;
    Recorder m;
    m.result = {2, -1, 0};
    m.ret = 2;
    const int n = search_for_initialization(m, F1, F2, prev, m12, 100);
    CHECK(n == 2 && m.orbdist == 100 && m.pos == (std::vector<float>{1, 2, 3, 4, 5, 6}));
    CHECK(m12 == (std::vector<int>{2, -1, 0}) && prev[1].x == 4.f && prev[2].y == 7.f);
  }

  if (g_fail) {
    std::printf("%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("OK adapter packers and appliers\n");
  return 0;
}
