"""The C3 step on one GPU, device-resident (BASELINE.json configs[2]): B stereo frames ->

  1. ORBextractor::operator() on all 2B images, lefts first   (ORBextractor.cc:1041-1103)
  (+ Frame::ComputeStereoMatches after extraction with stereo=True, Frame.cc:125)
  2. KeyFrame::ComputeBoW: TemplatedVocabulary::transform(desc, BowVector, FeatureVector, 4)
                                                              (KeyFrame.cc:59-68)
  3. ORBmatcher(0.6, false).SearchForTriangulation(KF1, KF2, F12, ..., false)
                                                              (LocalMapping.cc:219-258, ORBmatcher.cc:671-839)

Two pairings (`pairs`):
  "kf"      SURVEY 8(d)'s KeyFrame pairs: the B frames are consecutive frames of a driving sequence
            (orbfe_synth_sequence_frame, poses step_z apart along z), each a stereo KeyFrame whose
            keypoints and descriptors are the left image's (the stereo Frame's mvKeys,
            Frame.cc:113-130); ComputeBoW runs on the B lefts and SearchForTriangulation on
            (KF t, KF t+1) for t = 0..B-2 -- what LocalMapping::CreateNewMapPoints does for the new
            KeyFrame and its covisible predecessor (LocalMapping.cc:211-272). The epipole is the
            principal point, inside the image, so the epipole gate is live.
  "stereo"  the round-1/2 workload: ComputeBoW on all 2B images and SearchForTriangulation on
            (left_i, right_i) of one stereo frame (an x baseline: the epipole lies far outside).

bench.py times it and tests/test_gpu_c3.py checks it against the oracle, so both run this exact
sequence. The KeyFrames' per-keypoint state the matcher reads (mvuRight, GetMapPoint) is given
as device arrays `u_right` / `mp_state`, one `cap`-slot row per image.

Two output sets (depth 2) let sub-batch i's vocabulary + matching overlap sub-batch i+1's
extraction: extraction i -> matching i -> reuse of set i at sub-batch i + depth, ordered by
events on two streams.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib as L


def nodes_at_level_bound(tree, levelsup: int, cap: int) -> int:
    """Upper bound on FeatureVector entries: the nodes the descent can report at
    m_L - levelsup (nodes at that depth plus shallower leaves), capped by the feature count."""
    nid_level = tree.levels - levelsup
    if nid_level <= 0:
        return 1
    parent = tree.parent
    depth = np.zeros(len(parent), np.int32)
    par = np.maximum(parent, 0)
    for _ in range(tree.levels + 1):  # converges after the tree's depth
        depth[1:] = depth[par[1:]] + 1
    has_child = np.zeros(len(parent), bool)
    has_child[parent[1:]] = True
    n = int(((depth == nid_level) | ((depth < nid_level) & ~has_child & (depth > 0))).sum())
    return max(1, min(cap, n))


class DevEvent:
    """A cross-stream ordering event of the library (orbfe_event_create): no timing and no
    system-scope cache write-back on record, which a default (torch) event performs -- the
    pipeline's events only order device work between its streams; the host synchronises with
    torch.cuda.synchronize(). Same record(stream) / stream.wait_event(ev) interface as
    torch.cuda.Event."""

    def __init__(self, device: int):
        import ctypes
        p = ctypes.c_void_p()
        L.check(L.lib().orbfe_event_create(int(device), ctypes.byref(p)), "orbfe_event_create")
        self._e = p

    def record(self, stream) -> None:
        import ctypes
        L.check(L.lib().orbfe_event_record(self._e, ctypes.c_void_p(stream.cuda_stream)), "orbfe_event_record")

    def query(self) -> bool:
        """True when the recorded work is complete (hipEventQuery)."""
        r = L.lib().orbfe_event_query(self._e)
        L.check(min(r, 0), "orbfe_event_query")
        return r == 0

    def wait(self, stream) -> None:  # torch.cuda.Stream.wait_event(ev) calls ev.wait(stream)
        import ctypes
        L.check(L.lib().orbfe_stream_wait_event(ctypes.c_void_p(stream.cuda_stream), self._e),
                "orbfe_stream_wait_event")

    def __del__(self):
        try:
            if self._e:
                L.lib().orbfe_event_destroy(self._e)
        except Exception:  # interpreter shutdown
            pass


def new_event(device: int):
    """An ordering event for the pipeline's cross-stream dependencies: a DevEvent (torch's timing-
    capable events with their system-scope fence measured 0.6 % slower)."""
    return DevEvent(device)


class PipelineStreams:
    """The pipeline's concurrently busy streams, created natively in one go: one extraction stream
    per extractor, the matching stream, and (several extractors) one high-priority side stream
    they share. The runtime spreads streams over GPU_MAX_HW_QUEUES hardware queues per priority
    (4 by default), each new stream taking the least-shared queue and the first one on a tie, so
    the queue a stream lands on depends on every stream the process created before it; two busy
    streams on one queue serialise (measured on MI355X: 35.2k instead of 68.9k stereo frames/s
    after two idle streams had been created in between). Created before any other stream of the
    process, the busy streams each open a queue of their own."""

    def __init__(self, device: int, n_extractors: int = 1, match_inline: bool = False,
                 side_last: bool = False, comm: bool = False, copy: bool = False,
                 high=("side", "match")):
        import torch
        self.device = device
        self._ptrs = []
        self._attached = []

        def make(high):
            p = ctypes.c_void_p()
            L.check(L.lib().orbfe_stream_create(device, 1 if high else 0, ctypes.byref(p)), "stream_create")
            self._ptrs.append(p.value)
            return torch.cuda.ExternalStream(p.value, device=torch.device("cuda", device))

        n = max(1, n_extractors)
        # `high`: the streams created at high priority (the runtime serves each priority from its own
        # hardware queues); default the shared side stream and the matching stream
        self.extract = [make("extract" in high) for _ in range(n)]
        # the matching stream at high priority, beside the shared side stream, so that the
        # latency-bound vocabulary + SFT chain keeps up with the extraction handles (normal priority
        # and the other placements measured slower: DESIGN.md section 5); match_inline: each
        # sub-batch's vocabulary + matching follow its extraction on the same stream instead
        self.match = None
        if not match_inline and side_last:
            self.match = make("match" in high)
        self.side = make("side" in high)
        if not match_inline and not side_last:
            self.match = make("match" in high)
        # comm: a stream for the C4 gather's transfers, created here with the others so that it gets
        # a hardware queue of its own. A stream from torch's pool shares a queue with a pipeline
        # stream, and its barrier packets (waiting for the pack on the matching stream) then hold
        # that stream's kernels: measured 83k -> 52k stereo frames/s on one GPU (--gather-proxy)
        self.comm = make(False) if comm else None
        # copy: the H2D stream of a host-fed pipeline (bench.py --feed host), created last; with
        # more hardware queues than busy streams (the caller sets GPU_MAX_HW_QUEUES) it gets a queue
        # of its own, so that its waits for free input slots never hold an extraction stream
        self.copy = make(False) if copy else None

    def ordered(self):
        """(extraction streams..., matching stream or None) as C3Pipeline takes them."""
        return self.extract + [self.match]

    def attach(self, ext) -> None:
        """Route `ext`'s side-stream work to the shared side stream; detached again by close()."""
        ext.set_side_stream(self.side.cuda_stream)
        self._attached.append(ext)

    def close(self):
        """Wait for the streams, point every attached extractor back at its own side stream, then
        destroy the streams (no handle is left holding a destroyed hipStream_t)."""
        for s in self.extract + [self.match, self.comm, self.copy, self.side]:
            if s is not None:
                s.synchronize()
        for e in self._attached:
            e.set_side_stream(0)
        self._attached = []
        for p in self._ptrs:
            L.lib().orbfe_stream_destroy(ctypes.c_void_p(p))
        self._ptrs = []


class C3Pipeline:
    def __init__(self, ext, voc, tree, B: int, H: int, W: int, cam: dict, F12: np.ndarray,
                 epipole: tuple, grid_inv: tuple, mb: float, u_right, mp_state, device,
                 depth: int = 2, levelsup: int = 4, stereo: bool = False, bow: bool = True,
                 nnratio: float = 0.6, check_ori: bool = False, streams=None, pairs: str = "stereo",
                 stereo_on_match: bool = False, native: bool = True):
        import torch
        from .matcher import ORBmatcher
        # one extractor, or several whose extractions of consecutive sub-batches overlap on their
        # own streams (each keeps its own scratch)
        self.exts = list(ext) if isinstance(ext, (list, tuple)) else [ext]
        ext = self.exts[0]
        depth = max(depth, len(self.exts) + 1)
        self.ext, self.voc = ext, voc
        self.B, self.H, self.W = B, H, W
        self.n_img = 2 * B
        assert pairs in ("kf", "stereo")
        self.pairs_mode = pairs
        # images with a BowVector / FeatureVector, SearchForTriangulation pairs (kf1, kf2) per sub-batch
        self.n_vocab = B if pairs == "kf" else 2 * B
        self.pair_idx = [(i, i + 1) for i in range(B - 1)] if pairs == "kf" else [(i, B + i) for i in range(B)]
        self.n_pairs = len(self.pair_idx)
        n_pairs = self.n_pairs
        self.cap = cap = ext.max_keypoints(H, W)
        self.levelsup = levelsup
        self.stereo = stereo
        self.bow = bow
        self.mb = float(mb)
        self.cam = cam
        self.dev = dev = torch.device("cuda", device) if isinstance(device, int) else device
        self.d_ur, self.d_mp = u_right, mp_state
        self.d_scale = torch.from_numpy(ext.GetScaleFactors()).to(dev)
        self.d_sigma2 = torch.from_numpy(ext.GetScaleSigmaSquares()).to(dev)
        self.node_bound = nodes_at_level_bound(tree, levelsup, cap)
        n_img = self.n_img
        pipe = self

        class OutSet:
            def __init__(self):
                self.kps = torch.empty(n_img * cap * 28, dtype=torch.uint8, device=dev)
                self.desc = torch.empty(n_img * cap * 32, dtype=torch.uint8, device=dev)
                self.cnt = torch.zeros(n_img, dtype=torch.int32, device=dev)
                self.ids = torch.empty(n_img * cap, dtype=torch.int32, device=dev)
                self.offs = torch.empty(n_img * (cap + 1), dtype=torch.int32, device=dev)
                self.idx = torch.empty(n_img * cap, dtype=torch.int32, device=dev)
                self.nodes = torch.zeros(n_img, dtype=torch.int32, device=dev)
                self.bow_words = torch.empty(n_img * cap, dtype=torch.int32, device=dev)
                self.bow_weights = torch.empty(n_img * cap, dtype=torch.float64, device=dev)
                self.bow_n = torch.zeros(n_img, dtype=torch.int32, device=dev)
                self.m12 = torch.empty(max(n_pairs, 1) * cap, dtype=torch.int32, device=dev)
                self.nm = torch.zeros(max(n_pairs, 1), dtype=torch.int32, device=dev)
                self.ur = torch.full((B * cap,), -1.0, dtype=torch.float32, device=dev)
                self.dep = torch.full((B * cap,), -1.0, dtype=torch.float32, device=dev)
                self.matcher = ORBmatcher(nnratio, check_ori, device=dev.index)
                self.pairs = (L.sft_pair * max(n_pairs, 1))()
                for i, (a, b) in enumerate(pipe.pair_idx):
                    p = self.pairs[i]
                    p.kf1, p.kf2 = self.view(a), self.view(b)
                    p.fv1, p.fv2 = self.fvec(a), self.fvec(b)
                    for k, x in enumerate(np.asarray(F12, np.float32).reshape(9)):
                        p.f12[k] = float(x)
                    p.ex, p.ey = epipole
                    p.match12 = self.m12.data_ptr() + i * cap * 4
                    p.nmatches = self.nm.data_ptr() + i * 4
                    p.kf1_n_dev = self.cnt.data_ptr() + a * 4
                    p.kf2_n_dev = self.cnt.data_ptr() + b * 4
                    p.fv1_nodes_dev = self.nodes.data_ptr() + a * 4
                    p.fv2_nodes_dev = self.nodes.data_ptr() + b * 4
                self.extracted = new_event(dev.index)
                self.matched = new_event(dev.index)
                # set by an after_match hook whose work on another stream still reads the set (the
                # C4 gather): the set is reused only after it as well
                self.released = None
                self.mstream = None  # the stream the last matching of this set ran on

            def view(self, i):
                v = L.frame_view()
                v.n = 0  # read on the device from cnt[i]
                v.keys_un = self.kps.data_ptr() + i * cap * 28
                # left keyframes take mvuRight from ComputeStereoMatches when it runs
                v.u_right = (self.ur.data_ptr() + i * cap * 4 if stereo and i < B
                             else pipe.d_ur.data_ptr() + i * cap * 4)
                v.descriptors = self.desc.data_ptr() + i * cap * 32
                v.mp_state = pipe.d_mp.data_ptr() + i * cap
                v.nlevels = len(pipe.d_scale)
                v.scale_factors = pipe.d_scale.data_ptr()
                v.level_sigma2 = pipe.d_sigma2.data_ptr()
                v.min_x, v.max_x, v.min_y, v.max_y = 0.0, float(W), 0.0, float(H)
                v.grid_inv_w, v.grid_inv_h = float(grid_inv[0]), float(grid_inv[1])
                v.fx, v.fy, v.cx, v.cy, v.bf = cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["bf"]
                v.b = float(mb)
                return v

            def fvec(self, i):
                f = L.feature_vector()
                f.n_nodes = pipe.node_bound  # upper bound; the count is read on the device
                f.node_ids = self.ids.data_ptr() + i * cap * 4
                f.offsets = self.offs.data_ptr() + i * (cap + 1) * 4
                f.indices = self.idx.data_ptr() + i * cap * 4
                return f

        self.sets = [OutSet() for _ in range(max(1, depth))]
        self.lib = L.lib()
        # extraction (+ ComputeStereoMatches), default priority: giving it the side stream's high
        # priority measured 64.3k vs 69.6k stereo frames/s (MI355X)
        # `streams` = (one extraction stream per extractor, the matching stream), or a
        # PipelineStreams the caller created before anything else (hardware-queue assignment)
        if isinstance(streams, PipelineStreams):
            for e in self.exts:
                streams.attach(e)
            streams = streams.ordered()
        if streams is None:
            streams = [torch.cuda.Stream(dev) for _ in range(len(self.exts) + 1)]
        # several handles may share an extraction stream (handle k on stream k mod S): a handle's
        # pyramids are then rebuilt only every len(exts) sub-batches
        assert len(streams) >= 2 and len(self.exts) % (len(streams) - 1) == 0, \
            "the extractor count must be a multiple of the extraction streams"
        self.streams = list(streams[:-1])
        self.stream = self.streams[0]
        # vocabulary + matching (+ gather); None: on each sub-batch's extraction stream
        self.match_inline = streams[-1] is None
        self.mstream = self.stream if self.match_inline else streams[-1]
        self.counter = 0
        self.last = None
        self.last_stream = None
        self._torch = torch
        # stereo_on_match: ComputeStereoMatches on the matching stream (it needs only the extracted
        # pyramids and keypoints) instead of right after the extraction; the handle's next
        # extraction waits for it (run()). Measured on MI355X: with one handle per extraction
        # stream no gain (73.6-73.8k vs 74.2-76.5k stereo frames/s, round 3), with two handles per
        # stream -- the bench's shape, a handle's pyramids rebuilt only every fourth sub-batch --
        # 78.4-78.5k vs 77.1-77.5k, so bench.py turns it on (its --stereo-on-extract turns it off);
        # the class default stays off for single-handle callers
        self.stereo_on_match = stereo and stereo_on_match and not self.match_inline
        self.stereo_done = [None] * len(self.exts)
        # native: each sub-batch enqueued by one orbfe_c3_run call (include/orbfe_c3.h: the waits,
        # the extraction, ComputeStereoMatches, the vocabulary transform, SearchForTriangulation and
        # the ordering events from C++); otherwise the per-stage calls of run_stages() below.
        # Same work, same streams, same order.
        self._c3 = None
        if native:
            self._c3 = self._create_native()

    def _create_native(self):
        L_ = self.lib
        cfg = L.c3_config(n_images=self.n_img, rows=self.H, cols=self.W, cap=self.cap, n_vocab=self.n_vocab,
                          levelsup=self.levelsup, n_stereo=self.B if self.stereo else 0, mbf=float(self.cam["bf"]),
                          mb=self.mb, stereo_on_match=1 if self.stereo_on_match else 0, n_pairs=self.n_pairs)
        sets = (L.c3_set * len(self.sets))()
        for i, o in enumerate(self.sets):
            c = sets[i]
            c.kps, c.desc, c.counts = o.kps.data_ptr(), o.desc.data_ptr(), o.cnt.data_ptr()
            c.fv_node_ids, c.fv_offsets = o.ids.data_ptr(), o.offs.data_ptr()
            c.fv_indices, c.fv_n_nodes = o.idx.data_ptr(), o.nodes.data_ptr()
            if self.bow:
                c.bow_words, c.bow_weights, c.bow_n = (o.bow_words.data_ptr(), o.bow_weights.data_ptr(),
                                                       o.bow_n.data_ptr())
            if self.stereo:
                c.u_right, c.depth = o.ur.data_ptr(), o.dep.data_ptr()
            c.matcher = o.matcher._h
            c.pairs = ctypes.cast(o.pairs, ctypes.c_void_p)
        exts = (ctypes.c_void_p * len(self.exts))(*[e._h for e in self.exts])
        strs = (ctypes.c_void_p * len(self.streams))(*[st.cuda_stream for st in self.streams])
        h = ctypes.c_void_p()
        L.check(L_.orbfe_c3_create(ctypes.byref(cfg), exts, len(self.exts), strs, len(self.streams),
                                   None if self.match_inline else ctypes.c_void_p(self.mstream.cuda_stream),
                                   self.voc._h, sets, len(self.sets), ctypes.byref(h)), "orbfe_c3_create")
        return h

    def close(self):
        """Destroy the native plan (waits for its events); the buffers stay the caller's."""
        if getattr(self, "_c3", None):
            self.lib.orbfe_c3_destroy(self._c3)
            self._c3 = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def next_handle(self):
        """The extractor handle the next run() extracts with."""
        return self.exts[self.counter % len(self.exts)]

    def run(self, d_img_ptr: int, after_match=None, input_ready=None):
        """One sub-batch: 2B images of H x W at d_img_ptr (lefts then rights, row pitch W).
        `after_match(o)` runs on the matching stream after SearchForTriangulation (the C4 gather).
        `input_ready`: an event the extraction waits for first (the images' H2D copy of a host-fed
        pipeline). Returns the output set."""
        if self._c3 is not None:
            return self._run_native(d_img_ptr, after_match, input_ready)
        return self.run_stages(d_img_ptr, after_match, input_ready)

    def _run_native(self, d_img_ptr: int, after_match=None, input_ready=None):
        si = self.counter % len(self.sets)
        o = self.sets[si]
        k = self.counter % len(self.exts)
        self.counter += 1
        s = self.streams[k % len(self.streams)]
        L.check(self.lib.orbfe_c3_run(self._c3, si, k, ctypes.c_void_p(d_img_ptr),
                                      input_ready._e if input_ready is not None else None,
                                      1 if after_match is not None else 0), "orbfe_c3_run")
        o.ext, o.k = self.exts[k], k
        o.mstream = s if self.match_inline else self.mstream
        self.last_stream = s
        self.last = o
        if self.match_inline:
            self.mstream = s
        if after_match is not None:  # the C4 pack + gather on the matching stream, then the set's event
            o.released = None
            after_match(o)
            L.check(self.lib.orbfe_c3_finish(self._c3, si, o.released._e if o.released is not None else None),
                    "orbfe_c3_finish")
        return o

    def run_stages(self, d_img_ptr: int, after_match=None, input_ready=None):
        """run() as separate library calls per stage (the native plan's sequence, from Python)."""
        o = self.sets[self.counter % len(self.sets)]
        k = self.counter % len(self.exts)
        self.counter += 1
        B, H, W, cap = self.B, self.H, self.W, self.cap
        s, ext = self.streams[k % len(self.streams)], self.exts[k]
        if input_ready is not None:
            s.wait_event(input_ready)
        s.wait_event(o.matched)  # the matching that last read this set is done
        if o.released is not None:  # and whatever an after_match hook still runs on it (the gather)
            s.wait_event(o.released)
        if self.stereo_on_match and self.stereo_done[k] is not None:
            # ComputeStereoMatches of this handle's previous sub-batch (matching stream) read the
            # pyramids this extraction overwrites
            s.wait_event(self.stereo_done[k])
        ext.extract_batch_device(self.n_img, d_img_ptr, H * W, H, W, W, o.kps.data_ptr(),
                                 o.desc.data_ptr(), cap, o.cnt.data_ptr(), stream=s.cuda_stream)
        o.ext = ext
        o.k = k
        self.last_stream = s  # the extraction stream of this sub-batch
        if self.stereo and not self.stereo_on_match:  # Frame.cc:125, on the extraction stream
            self._stereo(o, ext, s)
        o.extracted.record(s)
        self.last = o
        if self.match_inline:
            self.mstream = s
        self._match(o, after_match)
        return o

    def _stereo(self, o, ext, stream):
        """Frame::ComputeStereoMatches (Frame.cc:125) of the set's B pairs on `stream`, from the
        pyramids handle `ext` built for it."""
        B, cap = self.B, self.cap
        ext.compute_stereo_matches_batch_device(B, 0, B, o.kps.data_ptr(), o.desc.data_ptr(),
                                                o.cnt.data_ptr(), cap, self.cam["bf"], self.mb,
                                                o.ur.data_ptr(), o.dep.data_ptr(), stream=stream.cuda_stream)

    def _match(self, o, after_match):
        B, cap = self.B, self.cap
        m = o.mstream = self.mstream
        if not self.match_inline:
            m.wait_event(o.extracted)
        if self.stereo and self.stereo_on_match:
            # off the extraction chain: the handle's next extraction waits for it (run())
            self._stereo(o, o.ext, m)
            if self.stereo_done[o.k] is None:  # one per handle, re-recorded (earlier waits keep the old record)
                self.stereo_done[o.k] = new_event(self.dev.index)
            self.stereo_done[o.k].record(m)
        self._vocab(o, m)
        if self.n_pairs:
            L.check(self.lib.orbfe_search_for_triangulation_batch_device(
                o.matcher._h, self.n_pairs, ctypes.cast(o.pairs, ctypes.c_void_p), 0, ctypes.c_void_p(m.cuda_stream)),
                "sft batch")
        if after_match is not None:
            after_match(o)
        o.matched.record(m)

    def _vocab(self, o, m):
        """KeyFrame::ComputeBoW of the set's KeyFrame images (n_vocab: the B lefts, or all 2B) on
        stream m."""
        bow = (dict(d_bow_words=o.bow_words.data_ptr(), d_bow_weights=o.bow_weights.data_ptr(),
                    d_bow_n=o.bow_n.data_ptr()) if self.bow else {})
        self.voc.transform_batch_device(self.n_vocab, o.desc.data_ptr(), self.cap * 32, o.cnt.data_ptr(),
                                        self.levelsup, o.ids.data_ptr(), o.offs.data_ptr(),
                                        o.idx.data_ptr(), o.nodes.data_ptr(), self.cap,
                                        stream=m.cuda_stream, **bow)

    def to_host(self, o=None) -> dict:
        """Every output of a sub-batch, per image / pair, as numpy (synchronises)."""
        import torch
        o = o or self.last
        torch.cuda.synchronize()
        cap, B = self.cap, self.B
        K = o.kps.cpu().numpy().view(L.KEYPOINT_DTYPE).reshape(self.n_img, cap)
        D = o.desc.cpu().numpy().reshape(self.n_img, cap, 32)
        C = o.cnt.cpu().numpy()
        I = o.ids.cpu().numpy().view(np.uint32).reshape(self.n_img, cap)
        OF = o.offs.cpu().numpy().reshape(self.n_img, cap + 1)
        X = o.idx.cpu().numpy().reshape(self.n_img, cap)
        NN = o.nodes.cpu().numpy()
        BW = o.bow_words.cpu().numpy().view(np.uint32).reshape(self.n_img, cap)
        BT = o.bow_weights.cpu().numpy().reshape(self.n_img, cap)
        BN = o.bow_n.cpu().numpy()
        M = o.m12.cpu().numpy().reshape(-1, cap)
        NM = o.nm.cpu().numpy()[:self.n_pairs]
        out = {"keypoints": [], "descriptors": [], "fv": [], "bow": [], "match12": [], "nmatches": NM.copy()}
        for i in range(self.n_img):
            n = int(C[i])
            out["keypoints"].append(K[i, :n].copy())
            out["descriptors"].append(D[i, :n].copy())
            if i >= self.n_vocab:
                continue
            k = int(NN[i])
            out["fv"].append((I[i, :k].copy(), OF[i, :k + 1].copy(), X[i, :OF[i, k]].copy()))
            nb = int(BN[i]) if self.bow else 0
            out["bow"].append((BW[i, :nb].copy(), BT[i, :nb].copy()))
        for p, (a, _) in enumerate(self.pair_idx):
            out["match12"].append(M[p, :int(C[a])].copy())
        if self.stereo:
            UR = o.ur.cpu().numpy().reshape(B, cap)
            out["u_right"] = [UR[p, :int(C[p])].copy() for p in range(B)]
        return out


STEP_Z = 1.0  # metres between consecutive frames of the C3 driving sequence


def build_c3(ext, tree, voc, B: int, H: int, W: int, device, seed: int = 1234, depth: int = 2,
             stereo: bool = False, levelsup: int = 4, streams=None, pairs: str = "stereo",
             stereo_on_match: bool = False, native: bool = True):
    """The C3 scene of bench.py: KITTI intrinsics, seeded KeyFrame state per keypoint slot (half
    the keypoints stereo unless ComputeStereoMatches provides mvuRight, 30 % with a MapPoint), and
    the KeyFrame pair geometry with F12 and epipole from LocalMapping::ComputeF12
    (LocalMapping.cc:545-561): pairs="kf" -- frame t and t+1 of the driving sequence, STEP_Z
    apart along z (epipole = principal point); pairs="stereo" -- the two cameras of one frame
    (t2 = -0.537 m, 0.05 m forward). Returns (pipeline, state) with state holding the host copies
    the oracle check needs."""
    import torch
    from . import synthetic as S
    from .frames import epipole as epipole_of
    dev = torch.device("cuda", device) if isinstance(device, int) else device
    exts = ext
    ext = exts[0] if isinstance(exts, (list, tuple)) else exts
    n_img = 2 * B
    cap = ext.max_keypoints(H, W)
    rng = np.random.default_rng(seed)
    ur = np.where(rng.random((n_img, cap)) < 0.5, rng.uniform(10, W - 41, (n_img, cap)), -1.0)
    ur = ur.astype(np.float32)
    mp = np.where(rng.random((n_img, cap)) < 0.3, L.ORBFE_MP_OBSERVED, L.ORBFE_MP_NONE).astype(np.uint8)
    cam = S.KITTI_CAM
    t1, t2 = (S.pose(), S.pose(tz=-STEP_Z)) if pairs == "kf" else (S.pose(), S.pose(tx=-0.537, tz=0.05))
    F12 = S.compute_f12(t1, t2, S.intrinsics(cam))
    scale, sigma2 = ext.GetScaleFactors(), ext.GetScaleSigmaSquares()
    dummy = S.make_frame(np.zeros(0, L.KEYPOINT_DTYPE), None, scale, sigma2, H, W, cam, rng, tcw=t1)
    dummy2 = S.make_frame(np.zeros(0, L.KEYPOINT_DTYPE), None, scale, sigma2, H, W, cam, rng, tcw=t2)
    ex, ey = epipole_of(dummy, dummy2)
    pipe = C3Pipeline(exts, voc, tree, B, H, W, cam, F12, (ex, ey),
                      (float(dummy.grid_inv_w), float(dummy.grid_inv_h)), float(dummy.mb),
                      torch.from_numpy(ur).to(dev), torch.from_numpy(mp).to(dev), dev, depth=depth,
                      levelsup=levelsup, stereo=stereo, streams=streams, pairs=pairs,
                      stereo_on_match=stereo_on_match, native=native)
    state = dict(u_right=ur, mp_state=mp, scale=scale, sigma2=sigma2, cam=cam, F12=F12,
                 epipole=(ex, ey), mb=float(dummy.mb), levelsup=levelsup, stereo=stereo, pairs=pairs)
    return pipe, state
