/*
 * orbfe.h -- C ABI of the MI355X-native ORB front-end (liborbfe.so).
 *
 * This is the drop-in boundary for ORB-SLAM2's per-frame feature path. Every entry point below
 * replaces one reference interface (cited file:line into lreithmayr/ORB_SLAM2_2021):
 *
 *   orbfe_extractor_create / _destroy   ORBextractor::ORBextractor          include/ORBextractor.h:56-57,
 *                                                                            src/ORBextractor.cc:413-473
 *   orbfe_get_scale_tables              ORBextractor::GetScaleFactors & co.  include/ORBextractor.h:70-98
 *   orbfe_extract                       ORBextractor::operator()             include/ORBextractor.h:66-68,
 *                                                                            src/ORBextractor.cc:1041-1103
 *   orbfe_extract_batch(_device)        N independent operator() calls (Frame.cc:113-116 runs two at once)
 *   orbfe_get_level                     public ORBextractor::mvImagePyramid  include/ORBextractor.h:100
 *   orbfe_descriptor_distance(_batch)   ORBmatcher::DescriptorDistance       src/ORBmatcher.cc:1672-1688
 *   orbfe_search_by_projection_local    ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
 *                                                                            src/ORBmatcher.cc:45-133
 *   orbfe_search_by_projection_lastframe ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 *                                                                            src/ORBmatcher.cc:1348-1491
 *   orbfe_search_for_triangulation      ORBmatcher::SearchForTriangulation   src/ORBmatcher.cc:671-839
 *
 * Conventions: plain pointers and sizes only; no C++ or torch types. Every function returns an int
 * status (ORBFE_OK = 0, negative on error) and never throws. Functions without the _device suffix
 * take HOST pointers and are synchronous. _device functions take DEVICE pointers, enqueue on the
 * given hipStream_t (passed as void*, NULL = the handle's own stream) and return immediately.
 * A handle is thread-compatible (one thread at a time), not thread-safe, mirroring one
 * ORBextractor instance per thread (Frame.cc:113-116).
 */
#ifndef ORBFE_H
#define ORBFE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBFE_OK 0
#define ORBFE_ERR_ARG -1       /* invalid argument (null pointer, bad size, unsupported geometry) */
#define ORBFE_ERR_CAPACITY -2  /* caller buffer too small; *n holds the required count */
#define ORBFE_ERR_HIP -3       /* HIP runtime error (message via orbfe_last_error) */
#define ORBFE_ERR_STATE -4     /* call order violated (e.g. get_level before any extract) */

#define ORBFE_DESC_BYTES 32

/* cv::KeyPoint field order: pt.x, pt.y, size, angle, response, octave, class_id (28 bytes). */
typedef struct orbfe_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbfe_keypoint;

typedef struct orbfe_extractor orbfe_extractor;

/* Pyramid vertical-rounding mode: OpenCV's x86 SIMD128 form on the columns
 * its 16/8-lane loops cover (the default build of OpenCV 4.5.x), or the scalar form everywhere. */
#define ORBFE_RESIZE_SIMD128 0
#define ORBFE_RESIZE_SCALAR 1

/* ---- extractor ---------------------------------------------------------------------------- */

/* ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) on HIP device `device`. */
int orbfe_extractor_create(int nfeatures, float scale_factor, int nlevels, int ini_th_fast,
                           int min_th_fast, int device, orbfe_extractor** out);
int orbfe_extractor_destroy(orbfe_extractor* h);
/* Select the resize rounding mode (default ORBFE_RESIZE_SIMD128). */
int orbfe_extractor_set_resize_mode(orbfe_extractor* h, int mode);

/* mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2 (nlevels floats each) and
 * mnFeaturesPerLevel (nlevels ints). Any pointer may be NULL. */
int orbfe_get_scale_tables(const orbfe_extractor* h, float* scale, float* inv_scale,
                           float* sigma2, float* inv_sigma2, int32_t* features_per_level);

/* Upper bound of keypoints one rows x cols image can produce: the sum over levels of
 * max(budget + 3, 4 * nIni) (an octree level may overshoot its budget by up to 3 in the refinement
 * loop, ORBextractor.cc:679-740, and its first pass yields up to 4 children per initial node).
 * Returns the bound (> 0) or a negative status. */
int orbfe_max_keypoints(orbfe_extractor* h, int rows, int cols);

/* operator()(image, mask, keypoints, descriptors) on one 8-bit grayscale image (host memory).
 * Writes *n keypoints (level order, ORBextractor.cc:1074-1102) and n x 32 descriptor bytes.
 * An empty image (rows == 0 or cols == 0) yields *n = 0 (ORBextractor.cc:1044-1045). */
int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int rows, int cols, size_t step,
                  orbfe_keypoint* kps, int cap, uint8_t* desc, int* n);

/* n_images independent operator() calls on same-shaped images (host memory). Image i starts at
 * imgs[i]; results for image i go to kps + i*cap, desc + i*cap*32, counts[i]. */
int orbfe_extract_batch(orbfe_extractor* h, int n_images, const uint8_t* const* imgs, int rows,
                        int cols, size_t step, orbfe_keypoint* kps, uint8_t* desc, int cap,
                        int32_t* counts);

/* Page-lock a caller buffer (hipHostRegister) that the host-buffer entry points then copy from /
 * to directly: images wholly inside registered ranges skip the pinned staging copy (runs of
 * images adjacent in memory go up in one DMA), and kps / desc inside registered ranges with
 * cap == orbfe_max_keypoints receive the results by DMA with no unpacking. Process-wide (any
 * handle, any device); a caller that reuses its image and keypoint buffers registers them once
 * (the reference's Frame keeps its cv::Mat images per frame; the adapter registers its ring of
 * frame buffers). Unregister before freeing the memory. Returns ORBFE_ERR_HIP if the runtime
 * refuses the range. */
int orbfe_host_register(const void* p, size_t bytes);
int orbfe_host_unregister(const void* p);

/* Device-resident batch: d_imgs holds n_images images, image i at d_imgs + i*image_stride, rows
 * `pitch` bytes apart. Outputs are device buffers laid out as in orbfe_extract_batch. Async on
 * `stream`. cap must be >= orbfe_max_keypoints(h). */
int orbfe_extract_batch_device(orbfe_extractor* h, int n_images, const uint8_t* d_imgs,
                               size_t image_stride, int rows, int cols, size_t pitch,
                               orbfe_keypoint* d_kps, uint8_t* d_desc, int cap,
                               int32_t* d_counts, void* stream);

/* Host view of pyramid level `level` of image `image` of the last extract call (mvImagePyramid,
 * read by Frame::ComputeStereoMatches, Frame.cc:529,620-640). The handle keeps one host copy per
 * image holding all its levels (rows `*step` bytes apart): the first access to an image copies
 * its whole pyramid in one DMA, unless the handle prefetched it (orbfe_extractor_set_host_pyramid).
 * Every level of every image of the call stays valid at once, until the next extract call on
 * this handle, as the reference's mvImagePyramid[0..nlevels-1] do. */
int orbfe_get_level(orbfe_extractor* h, int image, int level, const uint8_t** p, int* rows,
                    int* cols, size_t* step);

/* enable != 0: every later host-buffer extract call (orbfe_extract, orbfe_extract_batch) also
 * copies each image's pyramid to the handle's host block as soon as it is built, on a copy stream
 * beside the rest of the extraction, so orbfe_get_level returns without a copy. For callers that
 * read mvImagePyramid on the CPU after every call (the reference's Frame::ComputeStereoMatches).
 * Off by default: a GPU ComputeStereoMatches (orbfe_stereo.h) reads the device pyramids. */
int orbfe_extractor_set_host_pyramid(orbfe_extractor* h, int enable);

/* enable != 0: each extract call's launch sequence is captured into a hipGraph the first time its
 * arguments (images, outputs, stream, the handle's buffers and placement switches) are seen and
 * replayed with one graph launch afterwards (up to 8 argument sets per handle, least recently used
 * dropped); 0 (the default) launches every kernel directly. Same results either way. Measured on
 * MI355X / ROCm 7.2 the replay is slower: one 1241x376 image 0.33 vs 0.22 ms,
 * the C3 pipeline 38.6k vs 83.7k stereo frames/s. A handle whose side stream is a caller's shared
 * stream (orbfe_set_side_stream) always launches directly: a capture would pull that stream, which
 * other handles launch onto from their own threads, into the graph. */
int orbfe_extractor_set_graphs(orbfe_extractor* h, int enable);

/* Device pointer of the same level (no copy), for device-side consumers. */
int orbfe_get_level_device(orbfe_extractor* h, int image, int level, const uint8_t** d_p,
                           int* rows, int* cols, size_t* step);

/* Process-wide device-execution timing of the library's kernels (every handle, every thread).
 * orbfe_ktimer_select: comma-separated kernel names as rocprofv3 shows them without template
 * arguments ("k_fast,k_describe"), "*" for every kernel, "" or NULL for none. A selected launch
 * carries a start and a stop HIP event bound to the dispatch itself (hipExtLaunchKernelGGL), so
 * its time is the kernel's own execution interval -- what rocprofv3 --kernel-trace reports --
 * and excludes the queue's wait for earlier packets. orbfe_ktimer_read synchronises on the
 * pending launches and returns, per kernel timed since the process started (first-timed order),
 * the accumulated milliseconds and launch count; name_len bytes per name. ORBFE_ERR_CAPACITY
 * when more than `cap` kernels were timed (*n holds the count). orbfe_ktimer_reset zeroes the
 * totals. */
int orbfe_ktimer_select(const char* names);
int orbfe_ktimer_read(char* names, int name_len, double* total_ms, long long* launches, int cap,
                      int* n);
int orbfe_ktimer_reset(void);
/* The timer's own per-dispatch overhead: the median event interval of n launches of an empty
 * one-workgroup kernel on a private stream of `device`, in microseconds. The dispatch-bound events
 * include the dispatch's marker / launch latency beyond the kernel's execution, which rocprofv3's
 * kernel trace does not count; bench.py subtracts it per launch. */
int orbfe_ktimer_calibrate(int device, int n, double* overhead_us);

/* Stream the handle launches on (hipStream_t as void*). */
void* orbfe_extractor_stream(orbfe_extractor* h);

/* Event (hipEvent_t as void*) each launch sequence records on its stream as soon as the image
 * pyramid is complete (before FAST of the late levels, DistributeOctTree, the blur and the
 * descriptors). A caller that overlaps its own work with the extraction can order it after the
 * latency-bound pyramid phase: orbfe_stream_wait_event(its_stream, event) right after the
 * extract call, before the next one re-records the event. */
void* orbfe_extractor_pyramid_event(orbfe_extractor* h);
/* hipStreamWaitEvent(stream, event, 0) for callers without the HIP headers. */
int orbfe_stream_wait_event(void* stream, void* event);
/* An event (hipEvent_t as void*) that only orders device work between streams: no timing and no
 * system-scope release on record (hipEventDisableTiming | hipEventDisableSystemFence). A pipeline's
 * cross-stream dependencies recorded with it do not write the GPU caches back to memory each time,
 * which a default event does; nothing on the host may wait on it for data the device wrote.
 * orbfe_event_record = hipEventRecord(event, stream). */
int orbfe_event_create(int device, void** out);
int orbfe_event_record(void* event, void* stream);
/* 0: the event's work is complete (or it was never recorded), 1: not yet, < 0: error. */
int orbfe_event_query(void* event);
int orbfe_event_destroy(void* event);
/* A non-blocking stream on `device` (high_priority: the device's greatest priority, as the
 * extractor's side stream). The runtime maps streams onto a few hardware queues per priority
 * (GPU_MAX_HW_QUEUES, 4 by default), choosing the least-shared queue at creation and the
 * first queue on a tie; two busy streams that end up on one queue serialise. A caller that
 * runs several streams concurrently (e.g. extraction, side and matching streams of a
 * pipeline) creates them first, before any other stream, so that each takes its own queue. */
int orbfe_stream_create(int device, int high_priority, void** out);
int orbfe_stream_destroy(void* stream);
/* A stream whose kernels run only on the CUs set in cu_mask (n_words 32-bit words, bit i = CU i;
 * hipExtStreamCreateWithCUMask), normal priority: e.g. one half of the CUs per extractor handle. */
int orbfe_stream_create_masked(int device, const uint32_t* cu_mask, int n_words, void** out);

/* ---- matcher data (packed struct-of-arrays views of Frame / KeyFrame / MapPoint) ---------- */

/* MapPoint occupancy of a keypoint, from Frame::mvpMapPoints / KeyFrame::GetMapPoint:
 * NONE = NULL pointer; PRESENT = a MapPoint whose Observations() == 0; OBSERVED = Observations()>0. */
#define ORBFE_MP_NONE 0
#define ORBFE_MP_PRESENT 1
#define ORBFE_MP_OBSERVED 2

typedef struct orbfe_frame_view {
  int32_t n;                      /* Frame::N */
  const orbfe_keypoint* keys_un;  /* mvKeysUn */
  const float* u_right;           /* mvuRight (negative = no stereo) */
  const uint8_t* descriptors;     /* mDescriptors, n x 32 */
  const uint8_t* mp_state;        /* ORBFE_MP_* per keypoint */
  int32_t nlevels;
  const float* scale_factors;     /* mvScaleFactors */
  const float* level_sigma2;      /* mvLevelSigma2 */
  float min_x, max_x, min_y, max_y;  /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  float grid_inv_w, grid_inv_h;      /* mfGridElementWidthInv, mfGridElementHeightInv */
  float fx, fy, cx, cy, bf, b;       /* camera; bf = mbf, b = mb */
  /* KeyFrame views (orbfe_keyframe.h): the grid origin when it differs from min_x/min_y (the
   * Frame's float mnMinX/mnMinY that built mGrid; KeyFrame.h:202-205 keeps int bounds).
   * grid_origin_set = 0 (zero-initialised views): the grid origin is (min_x, min_y). */
  int32_t grid_origin_set;
  float grid_min_x, grid_min_y;
} orbfe_frame_view;

/* DBoW2::FeatureVector as CSR: node ids ascending, indices of node k in
 * indices[offsets[k] .. offsets[k+1]) in ascending feature order (TemplatedVocabulary.h:1161-1174). */
typedef struct orbfe_feature_vector {
  int32_t n_nodes;
  const uint32_t* node_ids;
  const int32_t* offsets;  /* n_nodes + 1 */
  const int32_t* indices;
} orbfe_feature_vector;

#define ORBFE_MPF_TRACK_IN_VIEW 1u  /* MapPoint::mbTrackInView */
#define ORBFE_MPF_BAD 2u            /* MapPoint::isBad() */
#define ORBFE_MPF_OBSERVED 4u       /* MapPoint::Observations() > 0 */
#define ORBFE_MPF_PRESENT 8u        /* LastFrame.mvpMapPoints[i] != NULL */
#define ORBFE_MPF_OUTLIER 16u       /* LastFrame.mvbOutlier[i] */

/* Local-map MapPoints as consumed by SearchByProjection(Frame&, vector<MapPoint*>, th). */
typedef struct orbfe_local_mappoints {
  int32_t m;
  const uint8_t* flags;        /* ORBFE_MPF_TRACK_IN_VIEW | _BAD | _OBSERVED */
  const float* proj_x;         /* mTrackProjX */
  const float* proj_y;         /* mTrackProjY */
  const float* proj_xr;        /* mTrackProjXR */
  const int32_t* level;        /* mnTrackScaleLevel */
  const float* view_cos;       /* mTrackViewCos */
  const uint8_t* descriptors;  /* GetDescriptor(), m x 32 */
} orbfe_local_mappoints;

/* Last frame's MapPoints as consumed by SearchByProjection(Frame&, const Frame&, th, bMono). */
typedef struct orbfe_lastframe_mappoints {
  int32_t n;                   /* LastFrame.N */
  const uint8_t* flags;        /* ORBFE_MPF_PRESENT | _OUTLIER | _OBSERVED */
  const float* world_pos;      /* GetWorldPos(), n x 3 */
  const uint8_t* descriptors;  /* GetDescriptor(), n x 32 */
  const int32_t* octave;       /* LastFrame.mvKeys[i].octave */
  const float* angle;          /* LastFrame.mvKeysUn[i].angle */
  float tcw_last[12];          /* LastFrame.mTcw rows 0..2 (3x4, row-major) */
} orbfe_lastframe_mappoints;

typedef struct orbfe_matcher orbfe_matcher;

/* ORBmatcher(nnratio, checkOri) bound to HIP device `device` (owns scratch + stream). */
int orbfe_matcher_create(float nnratio, int check_orientation, int device, orbfe_matcher** out);
int orbfe_matcher_destroy(orbfe_matcher* m);

/* DescriptorDistance over n pairs (host memory): out[i] = popcount(a_i xor b_i). */
int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b);
int orbfe_descriptor_distance_batch(orbfe_matcher* m, const uint8_t* a, const uint8_t* b, int n,
                                    int32_t* out);

/* SearchByProjection(F, vpMapPoints, th): best_idx[i] = keypoint index MapPoint i is assigned to
 * (F.mvpMapPoints[best_idx[i]] = vpMapPoints[i]; apply in ascending i), -1 if none.
 * *nmatches = the reference's return value. */
int orbfe_search_by_projection_local(orbfe_matcher* m, const orbfe_frame_view* frame,
                                     const orbfe_local_mappoints* mps, float th,
                                     int32_t* best_idx, int* nmatches);

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono): best_idx[i] for last-frame keypoint i:
 * -1 no match; k >= 0 CurrentFrame.mvpMapPoints[k] = LastFrame MapPoint i; k <= -2 the
 * assignment to keypoint (-2 - k) was made and then undone by the rotation-consistency filter
 * (ORBmatcher.cc:1469-1488): apply all assignments in ascending i, then NULL every undone
 * keypoint. tcw_cur = CurrentFrame.mTcw rows 0..2. */
int orbfe_search_by_projection_lastframe(orbfe_matcher* m, const orbfe_frame_view* current,
                                         const orbfe_lastframe_mappoints* last,
                                         const float* tcw_cur, float th, int mono,
                                         int32_t* best_idx, int* nmatches);

/* SearchForTriangulation(KF1, KF2, F12, pairs, bOnlyStereo): match12[idx1] = idx2 or -1;
 * the reference's pairs are (i, match12[i]) for ascending i with match12[i] >= 0.
 * f12: row-major 3x3 (F12.at<float>(r, c) = f12[3r + c]); (ex, ey) the epipole of KF1 in KF2
 * (ORBmatcher.cc:678-684). */
int orbfe_search_for_triangulation(orbfe_matcher* m, const orbfe_frame_view* kf1,
                                   const orbfe_frame_view* kf2, const orbfe_feature_vector* fv1,
                                   const orbfe_feature_vector* fv2, const float* f12, float ex,
                                   float ey, int only_stereo, int32_t* match12, int* nmatches);

/* Last error message of the calling thread (static storage). */
const char* orbfe_last_error(void);

/* Library build identity, e.g. "orbfe gfx950 <git>" */
const char* orbfe_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ORBFE_H */
