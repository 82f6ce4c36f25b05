// orbfe_c3.hip -- one call per C3 sub-batch (include/orbfe_c3.h): the extraction on a handle's
// stream, Frame::ComputeStereoMatches, KeyFrame::ComputeBoW and SearchForTriangulation on the
// matching stream, with the cross-stream ordering events, enqueued from C++ (host code only).
//
// Ordering per sub-batch (set o, handle k, extraction stream s, matching stream m):
//   s waits: input_ready, o.matched (the set's previous matching), o.released (an after-match
//            user of the set on another stream), stereo_done[k] (ComputeStereoMatches of k's
//            previous sub-batch read the pyramids this extraction overwrites)
//   s:       extraction (+ ComputeStereoMatches unless stereo_on_match), record o.extracted
//   m waits: o.extracted
//   m:       (ComputeStereoMatches, record stereo_done[k]), vocabulary transform,
//            SearchForTriangulation, record o.matched (or the caller does, orbfe_c3_finish)
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/orbfe.h"
#include "../../include/orbfe_c3.h"
#include "../../include/orbfe_match_batch.h"
#include "../../include/orbfe_stereo.h"
#include "../../include/orbfe_vocab.h"
#include "orbfe_device.h"

namespace {
constexpr unsigned kOrderEvent = hipEventDisableTiming | hipEventDisableSystemFence;

struct C3Set {
  orbfe_c3_set io;
  std::vector<orbfe_sft_pair> pairs;
  hipEvent_t extracted = nullptr, matched = nullptr;
  hipEvent_t released = nullptr;  // caller-owned
  hipStream_t mstream = nullptr;  // where its last matching ran
  int handle = 0;
};
}  // namespace

struct orbfe_c3 {
  orbfe_c3_config cfg{};
  int device = 0;
  std::vector<orbfe_extractor*> exts;
  std::vector<hipStream_t> streams;
  hipStream_t match = nullptr;
  orbfe_vocabulary* voc = nullptr;
  std::vector<C3Set> sets;
  std::vector<hipEvent_t> stereo_done;  // per handle
  std::vector<bool> stereo_recorded;
};

extern "C" int orbfe_c3_create(const orbfe_c3_config* cfg, orbfe_extractor* const* exts, int n_exts,
                               void* const* extract_streams, int n_streams, void* match_stream,
                               orbfe_vocabulary* voc, const orbfe_c3_set* sets, int n_sets, orbfe_c3** out) {
  if (!cfg || !exts || n_exts <= 0 || !extract_streams || n_streams <= 0 || n_exts % n_streams != 0 || !voc ||
      !sets || n_sets <= n_exts || !out || cfg->n_images <= 0 || cfg->rows <= 0 || cfg->cols <= 0 || cfg->cap <= 0 ||
      cfg->n_vocab < 0 || cfg->n_vocab > cfg->n_images || cfg->n_stereo < 0 || 2 * cfg->n_stereo > cfg->n_images ||
      cfg->n_pairs < 0)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_c3_create: bad argument");
  for (int i = 0; i < n_exts; i++)
    if (!exts[i]) return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_c3_create: null extractor");
  for (int i = 0; i < n_sets; i++) {
    const orbfe_c3_set& s = sets[i];
    if (!s.kps || !s.desc || !s.counts || (cfg->n_vocab > 0 && (!s.fv_node_ids || !s.fv_offsets || !s.fv_indices ||
                                                               !s.fv_n_nodes)) ||
        (cfg->n_stereo > 0 && (!s.u_right || !s.depth)) || (cfg->n_pairs > 0 && (!s.matcher || !s.pairs)))
      return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_c3_create: incomplete output set");
  }
  *out = nullptr;
  int dev = 0;
  ORBFE_HIP_CHECK(hipGetDevice(&dev));
  auto* c = new orbfe_c3();
  c->cfg = *cfg;
  c->device = dev;
  c->exts.assign(exts, exts + n_exts);
  for (int i = 0; i < n_streams; i++) c->streams.push_back((hipStream_t)extract_streams[i]);
  c->match = (hipStream_t)match_stream;
  c->voc = voc;
  c->sets.resize(n_sets);
  int st = ORBFE_OK;
  for (int i = 0; i < n_sets && st == ORBFE_OK; i++) {
    C3Set& s = c->sets[i];
    s.io = sets[i];
    if (cfg->n_pairs > 0) s.pairs.assign(sets[i].pairs, sets[i].pairs + cfg->n_pairs);
    s.io.pairs = nullptr;
    if (hipEventCreateWithFlags(&s.extracted, kOrderEvent) != hipSuccess ||
        hipEventCreateWithFlags(&s.matched, kOrderEvent) != hipSuccess)
      st = orbfe_set_error(ORBFE_ERR_HIP, "orbfe_c3_create: hipEventCreate");
  }
  c->stereo_done.assign(n_exts, nullptr);
  c->stereo_recorded.assign(n_exts, false);
  for (int k = 0; k < n_exts && st == ORBFE_OK; k++)
    if (hipEventCreateWithFlags(&c->stereo_done[k], kOrderEvent) != hipSuccess)
      st = orbfe_set_error(ORBFE_ERR_HIP, "orbfe_c3_create: hipEventCreate");
  if (st != ORBFE_OK) {
    orbfe_c3_destroy(c);
    return st;
  }
  *out = c;
  return ORBFE_OK;
}

static int c3_stereo(orbfe_c3* c, const C3Set& o, int k, hipStream_t s) {
  const orbfe_c3_config& g = c->cfg;
  return orbfe_compute_stereo_matches_batch_device(c->exts[k], g.n_stereo, 0, g.n_stereo, o.io.kps, o.io.desc,
                                                   o.io.counts, g.cap, g.mbf, g.mb, o.io.u_right, o.io.depth, s);
}

extern "C" int orbfe_c3_run(orbfe_c3* c, int set, int handle, const uint8_t* d_imgs, void* input_ready,
                            int defer_matched) {
  if (!c || set < 0 || set >= (int)c->sets.size() || handle < 0 || handle >= (int)c->exts.size() || !d_imgs)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_c3_run: bad argument");
  const orbfe_c3_config& g = c->cfg;
  C3Set& o = c->sets[set];
  const int k = handle;
  const hipStream_t s = c->streams[k % c->streams.size()];
  const bool stereo = g.n_stereo > 0, on_match = stereo && g.stereo_on_match && c->match;
  ORBFE_HIP_CHECK(hipSetDevice(c->device));
  if (input_ready) ORBFE_HIP_CHECK(hipStreamWaitEvent(s, (hipEvent_t)input_ready, 0));
  ORBFE_HIP_CHECK(hipStreamWaitEvent(s, o.matched, 0));  // (never recorded: no wait)
  if (o.released) ORBFE_HIP_CHECK(hipStreamWaitEvent(s, o.released, 0));
  if (on_match && c->stereo_recorded[k]) ORBFE_HIP_CHECK(hipStreamWaitEvent(s, c->stereo_done[k], 0));
  int st = orbfe_extract_batch_device(c->exts[k], g.n_images, d_imgs, (size_t)g.rows * g.cols, g.rows, g.cols,
                                      (size_t)g.cols, o.io.kps, o.io.desc, g.cap, o.io.counts, s);
  if (st != ORBFE_OK) return st;
  if (stereo && !on_match) {  // Frame.cc:125, on the extraction stream
    st = c3_stereo(c, o, k, s);
    if (st != ORBFE_OK) return st;
  }
  ORBFE_HIP_CHECK(hipEventRecord(o.extracted, s));
  const hipStream_t m = c->match ? c->match : s;
  if (c->match) ORBFE_HIP_CHECK(hipStreamWaitEvent(m, o.extracted, 0));
  if (on_match) {  // off the extraction chain; handle k's next extraction waits for it
    st = c3_stereo(c, o, k, m);
    if (st != ORBFE_OK) return st;
    ORBFE_HIP_CHECK(hipEventRecord(c->stereo_done[k], m));
    c->stereo_recorded[k] = true;
  }
  if (g.n_vocab > 0) {  // KeyFrame::ComputeBoW
    st = orbfe_vocab_transform_batch_device(c->voc, g.n_vocab, o.io.desc, (size_t)g.cap * 32, o.io.counts, g.levelsup,
                                            o.io.bow_words, o.io.bow_weights, o.io.bow_n, o.io.fv_node_ids,
                                            o.io.fv_offsets, o.io.fv_indices, o.io.fv_n_nodes, g.cap, m);
    if (st != ORBFE_OK) return st;
  }
  if (g.n_pairs > 0) {  // SearchForTriangulation(KF t, KF t+1) of every pair
    st = orbfe_search_for_triangulation_batch_device(o.io.matcher, g.n_pairs, o.pairs.data(), 0, m);
    if (st != ORBFE_OK) return st;
  }
  o.mstream = m;
  o.handle = k;
  o.released = nullptr;
  if (!defer_matched) ORBFE_HIP_CHECK(hipEventRecord(o.matched, m));
  return ORBFE_OK;
}

extern "C" int orbfe_c3_finish(orbfe_c3* c, int set, void* released) {
  if (!c || set < 0 || set >= (int)c->sets.size() || !c->sets[set].mstream)
    return orbfe_set_error(ORBFE_ERR_ARG, "orbfe_c3_finish: bad argument");
  C3Set& o = c->sets[set];
  ORBFE_HIP_CHECK(hipSetDevice(c->device));
  ORBFE_HIP_CHECK(hipEventRecord(o.matched, o.mstream));
  o.released = (hipEvent_t)released;
  return ORBFE_OK;
}

extern "C" void* orbfe_c3_match_stream(orbfe_c3* c, int set) {
  if (!c || set < 0 || set >= (int)c->sets.size()) return nullptr;
  return (void*)c->sets[set].mstream;
}

extern "C" int orbfe_c3_destroy(orbfe_c3* c) {
  if (!c) return ORBFE_OK;
  hipSetDevice(c->device);
  for (auto& s : c->sets) {
    if (s.extracted) hipEventSynchronize(s.extracted);
    if (s.matched) hipEventSynchronize(s.matched);
    if (s.extracted) hipEventDestroy(s.extracted);
    if (s.matched) hipEventDestroy(s.matched);
  }
  for (auto e : c->stereo_done)
    if (e) {
      hipEventSynchronize(e);
      hipEventDestroy(e);
    }
  delete c;
  return ORBFE_OK;
}
