// TEST-ONLY matcher for tests/cpp/matcher_tsan.cpp: orbfe::Matcher's signatures (include/orbfe.hpp)
// without a device. adapter/ORBmatcher_gpu.cc is compiled with ORBFE_ADAPTER_MATCHER=TsanMatcher
// and this header force-included, so the adapter's packers run under ThreadSanitizer on the CPU.
// Every search reads all of the views it is handed (so the sanitizer sees the packed arrays used)
// and returns "no match".
#ifndef ORBFE_TSAN_MATCHER_H
#define ORBFE_TSAN_MATCHER_H
#include <cstdint>
#include <utility>
#include <vector>

#include "orbfe.h"
#include "orbfe_keyframe.h"

struct TsanMatcher {
  TsanMatcher(float, bool) {}
  static unsigned touch(const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    unsigned s = 0;
    for (size_t i = 0; i < n; i++) s += b[i];
    return s;
  }
  static unsigned frame(const orbfe_frame_view& f) {
    return touch(f.keys_un, sizeof(orbfe_keypoint) * f.n) + touch(f.mp_state, f.n) + touch(f.descriptors, 32u * f.n);
  }
  static unsigned geo(const orbfe_mappoint_geometry& g) {
    return touch(g.flags, g.m) + touch(g.world_pos, 12u * g.m) + touch(g.normal, 12u * g.m) +
           touch(g.min_distance, 4u * g.m) + touch(g.max_distance, 4u * g.m) + touch(g.descriptors, 32u * g.m);
  }
  static int none(int n, std::vector<int32_t>& out) {
    out.assign(n > 0 ? n : 0, -1);
    return 0;
  }
  unsigned sink = 0;
  int SearchByProjection(const orbfe_frame_view& F, const orbfe_local_mappoints& m, float, std::vector<int32_t>& b) {
    sink += frame(F) + touch(m.flags, m.m) + touch(m.descriptors, 32u * m.m);
    return none(m.m, b);
  }
  int SearchByProjection(const orbfe_frame_view& c, const orbfe_lastframe_mappoints& l, const float*, float, bool,
                         std::vector<int32_t>& b) {
    sink += frame(c) + touch(l.flags, l.n) + touch(l.world_pos, 12u * l.n) + touch(l.descriptors, 32u * l.n);
    return none(l.n, b);
  }
  int SearchForTriangulation(const orbfe_frame_view& a, const orbfe_frame_view& b, const orbfe_feature_vector&,
                             const orbfe_feature_vector&, const float*, float, float,
                             std::vector<std::pair<size_t, size_t>>& pairs, bool) {
    sink += frame(a) + frame(b);
    pairs.clear();
    return 0;
  }
  int SearchByBoW(const orbfe_frame_view& k, const orbfe_feature_vector&, const orbfe_frame_view& f,
                  const orbfe_feature_vector&, std::vector<int32_t>& m) {
    sink += frame(k) + frame(f);
    return none(f.n, m);
  }
  int SearchByBoW12(const orbfe_frame_view& a, const orbfe_feature_vector&, const orbfe_frame_view& b,
                    const orbfe_feature_vector&, std::vector<int32_t>& m) {
    sink += frame(a) + frame(b);
    return none(a.n, m);
  }
  int SearchByProjection(const orbfe_frame_view& c, const float*, const orbfe_mappoint_geometry& g, const float*,
                         float, float, int, std::vector<int32_t>& b) {
    sink += frame(c) + geo(g);
    return none(g.m, b);
  }
  int SearchByProjectionSim3(const orbfe_frame_view& k, const float*, const orbfe_mappoint_geometry& g, float, int,
                             std::vector<int32_t>& b) {
    sink += frame(k) + geo(g);
    return none(g.m, b);
  }
  int Fuse(const orbfe_frame_view& k, const float*, const float*, const orbfe_mappoint_geometry& g, float, float,
           std::vector<int32_t>& b) {
    sink += frame(k) + geo(g);
    return none(g.m, b);
  }
  int FuseSim3(const orbfe_frame_view& k, const float*, const orbfe_mappoint_geometry& g, float, float,
               std::vector<int32_t>& b) {
    sink += frame(k) + geo(g);
    return none(g.m, b);
  }
  int SearchBySim3(const orbfe_frame_view& a, const orbfe_frame_view& b, const orbfe_mappoint_geometry& g1,
                   const orbfe_mappoint_geometry& g2, const float*, const float*, float, const float*, const float*,
                   float, float, float, std::vector<int32_t>& m) {
    sink += frame(a) + frame(b) + geo(g1) + geo(g2);
    return none(a.n, m);
  }
  int SearchForInitialization(const orbfe_frame_view& a, const orbfe_frame_view& b, std::vector<float>&,
                              std::vector<int32_t>& m, int) {
    sink += frame(a) + frame(b);
    return none(a.n, m);
  }
};
#endif
