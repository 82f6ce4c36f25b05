#!/usr/bin/env python3
"""Benchmark: ORB extract + match on synthetic 1241x376 KITTI-shaped stereo frames.

A step is one pass of the hot path over one batch of synthetic input resident in HBM: S
sub-batches (default 1024) of B = 32 stereo frames per GPU (BASELINE.json configs[2], "C3"), each
sub-batch (orb_slam2_2021_amd.pipeline.C3Pipeline):
  1. the stereo Frame constructor (Frame.cc:113-125): ORBextractor::operator() on its 2B images
     (k_copy0, k_resize x7, k_fast, k_octree, k_blur, k_describe), then Frame::ComputeStereoMatches
     (k_stereo_*) for the left KeyFrames' mvuRight
  2. KeyFrame::ComputeBoW of the B left KeyFrames: vocabulary transform, ORBvoc-shaped k=10/L=6
     tree, levelsup 4 (BowVector + FeatureVector; k_vocab_descend + k_vocab)
  3. ORBmatcher::SearchForTriangulation(KF t, KF t+1) for the B-1 consecutive KeyFrame pairs of the
     driving sequence, 1 m apart along z (k_sft_*)
  4. with N > 1 GPUs: the used keypoints + descriptors of every rank gathered to rank 0 over RCCL
     (config C4: packed on the device, fixed-count point-to-point payloads, no host sync)
--pairs stereo runs rounds 1-2's workload instead (ComputeBoW on all 2B images,
SearchForTriangulation(left_i, right_i) of one frame). The sub-batches cycle over --input-batches
(default 8) distinct resident batches, so no sub-batch re-reads the previous one's input.
value = stereo frames processed by all ranks / max-over-ranks wall time of the K timed steps.

Launch: python bench.py [--gpus N] [--steps K] [--warmup W]. With N > 1 and no torch.distributed
environment, the script starts torch.distributed.run as a child process (before any GPU call)
and exits with its status; the driver's own torchrun launch is used as is.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec (ORB extract+match) on 1241×376, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=32, help="stereo frames per GPU per sub-batch (C3)")
    p.add_argument("--batches-per-step", type=int, default=1024,
                   help="sub-batches per step: a step is long enough for external samplers to see")
    p.add_argument("--input-batches", type=int, default=8,
                   help="distinct HBM-resident input batches the sub-batches cycle over")
    p.add_argument("--rows", type=int, default=376)
    p.add_argument("--cols", type=int, default=1241)
    p.add_argument("--nfeatures", type=int, default=2000)
    p.add_argument("--vocab-levels", type=int, default=6, help="synthetic ORBvoc depth (k = 10)")
    p.add_argument("--levelsup", type=int, default=4, help="KeyFrame::ComputeBoW's levelsup")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="CPU baseline time per mode")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the all-core CPU baseline (0: the affinity mask, capped by OMP_NUM_THREADS)")
    p.add_argument("--event-every", type=int, default=16,
                   help="every kernel timed by dispatch-bound events on every n-th group of timed sub-batches "
                        "(every 4th group cost 2.2 %% of the value, every 8th 1.1 %%, round 4)")
    p.add_argument("--probe-subbatches", type=int, default=24,
                   help="with --no-kernel-events: sub-batches of the untimed pass that times every kernel")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-gather", action="store_true")
    p.add_argument("--no-kernel-events", action="store_true")
    p.add_argument("--no-legs", action="store_true", help="skip the secondary measurements")
    p.add_argument("--no-parity", action="store_true", help="skip the oracle check of the last sub-batch")
    p.add_argument("--pipeline", type=int, default=0,
                   help="output sets in flight (0: 2 per extractor handle; 1: strictly one at a time)")
    p.add_argument("--pairs", choices=("kf", "stereo"), default="kf",
                   help="SearchForTriangulation pairs: kf = KeyFrame t vs t+1 of a driving sequence (SURVEY 8(d); "
                        "ComputeBoW on the lefts), stereo = left vs right image of one frame (rounds 1-2)")
    p.add_argument("--no-stereo", dest="stereo", action="store_false",
                   help="skip Frame::ComputeStereoMatches (the stereo Frame constructor's matching, Frame.cc:125, "
                        "whose mvuRight feeds SearchForTriangulation; on by default)")
    p.add_argument("--extractors", type=int, default=2,
                   help="extractor handles whose extractions of consecutive sub-batches overlap, each on its "
                        "own stream, their side-stream work on one shared high-priority stream")
    p.add_argument("--handles-per-stream", type=int, default=2,
                   help="extractor handles per extraction stream (handle k on stream k mod --extractors): "
                        "a handle's pyramids are rebuilt every extractors x this sub-batches")
    p.add_argument("--hw-queues", type=int, default=-1,
                   help="GPU_MAX_HW_QUEUES for this process (set before the HIP runtime starts; 0: the "
                        "environment's, 4 by default; -1 (default): 8 when WORLD_SIZE > 1, so that the RCCL "
                        "stream of the C4 gather gets a queue of its own instead of sharing one with an "
                        "extraction stream, else the environment's): hardware queues the busy streams spread over")
    p.add_argument("--fast-side", type=int, default=4,
                   help="FAST of levels 0..K-1 on the extractor's side stream as each level is built "
                        "(0: the library default, levels 0..2, best with one handle; 4 with the pipeline's four "
                        "handles: 82.9k vs 82.0k stereo frames/s, interleaved, round 4)")
    p.add_argument("--diag-skip-matching", action="store_true",
                   help="diagnostic, not the metric: skip ComputeBoW + SearchForTriangulation (extraction-only rate)")
    p.add_argument("--inline-side", action="store_true",
                   help="diagnostic: every handle's side-stream work on its own launch stream (with "
                        "--extractors 1 --pipeline 1 every kernel runs alone)")
    p.add_argument("--blur-mode", type=int, default=-1,
                   help="GaussianBlur placement (orbfe_debug_set_blur_mode): 0 beside DistributeOctTree on the "
                        "side stream, 1 after it on the launch stream (default: 0 with one handle, 1 with several)")
    p.add_argument("--octree-split", type=int, default=-1,
                   help="DistributeOctTree launch split (orbfe_debug_set_octree_split): levels 0..K-1 at 80 KiB of "
                        "LDS per block, K.. at 40 KiB; 0: one launch (default: the library's, 5: 86.7-86.9k vs 85.7-85.9k "
                        "at 4 and 84.0-84.1k at 0, rounds 5-6)")
    p.add_argument("--fast-side-merge", action="store_true",
                   help="side-stream FAST levels 1..k-1 in one launch (orbfe_debug_set_fast_side_merge)")
    p.add_argument("--pyramid-tiles", default="",
                   help="k_pyramid tiles per image sx,sy,bx,by for calls of < 8 images / batches "
                        "(orbfe_debug_set_pyramid_tiles; 0,0: the per-level resize chain)")
    p.add_argument("--octree-threads", default="",
                   help="SMALL,BATCH: DistributeOctTree's block size for calls of < 8 images and for batches "
                        "(orbfe_debug_set_octree_threads; default 512,256)")
    p.add_argument("--octree-lds", default="",
                   help="HI,LO: LDS KiB per block of the two octree launches (orbfe_debug_set_octree_lds; "
                        "default: the library's 80,40)")
    p.add_argument("--fast-wpb", default="",
                   help="SIDE,MAIN: k_fast cells per workgroup of the side-stream / remaining launches "
                        "(orbfe_debug_set_fast_wpb; default: the library's 4,1)")
    p.add_argument("--high-prio", default="side,match",
                   help="pipeline streams created at high priority: any of extract, side, match (default side,match)")
    p.add_argument("--stage-calls", action="store_true",
                   help="enqueue each sub-batch stage by stage from Python (~25 library calls) instead of "
                        "one orbfe_c3_run call (include/orbfe_c3.h)")
    p.add_argument("--graphs", action="store_true",
                   help="replay each extraction's launch sequence from the handle's captured hipGraphs "
                        "(orbfe_extractor_set_graphs; off by default: 38.6k vs 83.7k stereo frames/s, round 5)")
    p.add_argument("--match-inline", action="store_true",
                   help="vocabulary + matching on each sub-batch's extraction stream (no matching stream)")
    p.add_argument("--stereo-on-extract", action="store_true",
                   help="ComputeStereoMatches on the extraction stream right after each extraction (rounds 1-3's "
                        "placement; default: on the matching stream ahead of the vocabulary, with two handles per "
                        "extraction stream so no extraction waits for it: 78.4-78.5k vs 77.1-77.5k)")
    p.add_argument("--dump-gather", default="",
                   help="test hook: write each rank's last sub-batch (own keypoints + descriptors) and "
                        "rank 0's gathered payloads to this directory")
    p.add_argument("--c5-workers", type=int, default=4,
                   help="C5 leg: Tracking-like callers per rank, each with its own extractor + matcher on its "
                        "own thread (the leg also reports one caller)")
    p.add_argument("--gather-every", type=int, default=1,
                   help="--gather-proxy: the packed payloads of K sub-batches per RCCL group")
    p.add_argument("--gather-proxy", type=int, default=0,
                   help="one-GPU proxy of C4's rank-0 ingestion at N GPUs: after each sub-batch's pack, "
                        "N-1 RCCL self send / receive pairs of the packed worst-case payload (a world-1 "
                        "communicator) as one group on the matching stream, where Gatherer's transfers run, "
                        "with N > 1's hardware-queue setting (DESIGN.md section 7)")
    p.add_argument("--feed", choices=("device", "host"), default="device",
                   help="device: the input batches resident in HBM when the timed region starts (the metric); "
                        "host: every sub-batch's 2B images copied from pinned host memory on a copy stream into "
                        "one of --input-slots device slots, overlapped with the other sub-batches' extraction and "
                        "matching (the reference's operator() takes host images, ORBextractor.cc:1041-1048)")
    p.add_argument("--copy-streams", type=int, default=1, choices=(1, 2),
                   help="--feed host: copy streams per sub-batch's H2D (2: two halves on two streams)")
    p.add_argument("--input-slots", type=int, default=0,
                   help="--feed host: device input slots (0: two per extractor handle)")
    p.add_argument("--copies-ahead", type=int, default=-1,
                   help="--feed host: copies enqueued this many sub-batches ahead of their extraction "
                        "(-1: (R - 1) / 2 of the R input slots; 0: each just before its extraction)")
    p.add_argument("--host-pin", choices=("torch", "register"), default="torch",
                   help="--feed host: page-lock the host images with torch's pin_memory (hipHostMalloc) or "
                        "register the numpy buffer in place (orbfe_host_register, hipHostRegister)")
    p.add_argument("--root-share", type=float, default=-1.0,
                   help="C4 (and --gather-proxy): the fraction of the per-rank sub-batches rank 0 extracts and "
                        "matches itself, since it also ingests every peer's payload; on the other slots it only "
                        "receives (-1: the model of DESIGN.md section 7, 1 - ROOT_INGEST_PER_PEER (N - 1))")
    p.add_argument("--rehearse", action="store_true",
                   help="N ranks on ONE GPU over gloo with host-staged exchanges: exercises the multi-rank "
                        "orchestration on a one-GPU box (not a measurement)")
    return p.parse_args(argv)


# N > 1: the C4 transfers run on the matching stream (Gatherer), but RCCL's own internal streams
# and torch.distributed's collective stream (the barrier / all-reduce around the timed region, the
# ORBFE_GATHER=torch path) come on top of the four busy pipeline streams. With the HIP default of 4
# hardware queues an extra busy stream shares a queue with a pipeline stream, and a receive kernel
# waiting for its peer then holds that queue (five busy streams on 4 queues measured 54.9k vs 78.9k
# stereo frames/s in round 2); 8 queues with two extraction streams measured the same as 4 at N = 1
HW_QUEUES_MULTI_RANK = 8

def hw_queue_setting(requested: int, world: int) -> int:
    """GPU_MAX_HW_QUEUES to set (0: leave the environment's): --hw-queues as given, or with the
    default (-1) HW_QUEUES_MULTI_RANK when this is one of several ranks."""
    if requested >= 0:
        return requested
    return HW_QUEUES_MULTI_RANK if world > 1 else 0


# C4: rank 0's cost of ingesting one peer's packed sub-batch payload, as a fraction of a sub-batch
# period, from the one-GPU proxy (--gather-proxy N: N - 1 RCCL self send / receive pairs per slot,
# the send side's HBM traffic included, so an upper bound): round 4 -2.5 / -11.6 / -19.1 % at
# N = 2 / 4 / 8 (2.7 % per peer); round 5, N = 8: 504.4 vs 387.6 ms per 1,024-sub-batch step, i.e.
# 116.8 ms for 7,168 payloads = 4.3 % of a period per payload (profiles/r5_c4_proxy.txt). The larger
# figure: if it overstates the cost, rank 0 finishes first and the whole job still loses only
# (1 - f) / N.
ROOT_INGEST_PER_PEER = 0.043


def root_share(requested: float, n_gpus: int) -> float:
    """Fraction of the per-rank sub-batch slots on which rank 0 runs its own sub-batch (it receives
    the peers' payloads on every slot). With rank 0 slower by c (N - 1) per own sub-batch, the ranks
    finish together when rank 0 runs 1 - c (N - 1) of the slots: frames = (N - 1 + f) S B in the
    peers' time S p, a whole-job loss of (1 - f) / N (2.4 % at N = 8) instead of c (N - 1) (19 %)."""
    if requested >= 0:
        return min(1.0, max(0.0, requested))
    if n_gpus <= 1:
        return 1.0
    return max(0.5, 1.0 - ROOT_INGEST_PER_PEER * (n_gpus - 1))


def own_slots(n: int, share: float):
    """Which of n slots run the rank's own sub-batch: round(n share) of them, spread evenly."""
    import math
    return [math.floor((k + 1) * share + 0.5) > math.floor(k * share + 0.5) for k in range(n)]


SEQ_SEED = 0x0C3  # the C3 driving sequence (orbfe_synth_sequence_frame)


def make_inputs(args, world, rank):
    """NB distinct batches of B stereo frames of this rank (frames sharded contiguously over the
    ranks, shard_frames): frames of the seeded driving sequence for --pairs kf (batch j holds
    consecutive frames, so KeyFrame t and t+1 are neighbours), independent seeded frames
    (orbfe_synth_frame) for --pairs stereo. Rendered on a thread pool (the C renderer releases the
    GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    from orb_slam2_2021_amd import synth_frame, synth_sequence_frame
    from orb_slam2_2021_amd.parallel import shard_frames
    B, H, W, NB = args.batch, args.rows, args.cols, max(1, args.input_batches)
    host = np.zeros((NB, 2 * B, H, W), np.uint8)
    mine = shard_frames(world * NB * B, world, rank)

    def one(ji):
        j, i = ji
        idx = mine[j * B + i]
        if args.pairs == "kf":
            host[j, i], host[j, B + i] = synth_sequence_frame(SEQ_SEED, idx, H, W, right=True)
        else:
            host[j, i], host[j, B + i] = synth_frame(idx, H, W, right=True)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as pool:
        list(pool.map(one, [(j, i) for j in range(NB) for i in range(B)]))
    return host


def spawn_ranks(args) -> int:
    """N > 1 without a torch.distributed environment: torchrun as a child process, one rank per
    GPU, over 127.0.0.1. This process has not touched the GPU (no HIP call before this point)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


class Gatherer:
    """C4: each sub-batch's used keypoints + descriptors to rank 0. The pack kernel runs on the
    matching stream right after SearchForTriangulation, and the point-to-point transfers of a fixed
    byte count (the packed worst case; the packed header carries the per-image counts) follow it on
    the same stream as one RCCL group (orb_slam2_2021_amd.rccl): no size exchange, so the host never
    waits for the device inside the timed loop, and no cross-stream event (an idle stream made to
    wait for the matching stream's pack every sub-batch cost 37 % of the throughput on one GPU,
    DESIGN.md section 7). The set's o.matched follows the transfers on the stream. ORBFE_GATHER=torch
    (and --rehearse) use torch.distributed's process group instead (parallel.gather_fixed on a comm
    stream that waits for the pack; o.released recorded behind the transfers)."""

    def __init__(self, pipe, world, rank, dev, comm_dev, comm=None):
        import torch
        from orb_slam2_2021_amd.parallel import packed_bytes
        self.pipe, self.world, self.rank = pipe, world, rank
        self.comm_dev = comm_dev  # the payload's device for the exchange (host only in --rehearse)
        self.cap_bytes = packed_bytes(pipe.n_img, pipe.n_img * pipe.cap)
        self.bufs = {id(o): torch.empty(self.cap_bytes, dtype=torch.uint8, device=dev) for o in pipe.sets}
        self.sizes = {id(o): torch.zeros(1, dtype=torch.int64, device=dev) for o in pipe.sets}
        self.recv = ([torch.empty(self.cap_bytes, dtype=torch.uint8, device=comm_dev) for _ in range(world)]
                     if rank == 0 else None)
        self.transfers = 0
        self.last = None  # rank 0: the last exchange's per-rank views (alias the receive buffers)
        self.last_set = None
        # the pipeline's comm stream (a hardware queue of its own, PipelineStreams)
        self.comm = comm if comm is not None else torch.cuda.Stream(dev)
        from orb_slam2_2021_amd.pipeline import new_event
        self.packed = {id(o): new_event(dev.index) for o in pipe.sets}
        self.sent = {id(o): new_event(dev.index) for o in pipe.sets}
        self.rccl = None
        if comm_dev.type != "cpu" and os.environ.get("ORBFE_GATHER", "rccl") == "rccl":
            from orb_slam2_2021_amd.rccl import RcclComm
            try:
                self.rccl = RcclComm.from_process_group()
            except (OSError, RuntimeError, AttributeError) as e:  # every rank fails alike (library / init)
                print(f"rank {rank}: RCCL communicator unavailable ({e}); C4 through torch.distributed",
                      file=sys.stderr)

    def pack(self, o):
        import torch
        from orb_slam2_2021_amd.parallel import gather_fixed, pack_keypoints_device
        p = self.pipe
        buf = self.bufs[id(o)]
        pack_keypoints_device(p.n_img, o.cnt.data_ptr(), o.kps.data_ptr(), o.desc.data_ptr(), p.cap,
                              buf.data_ptr(), self.cap_bytes, self.sizes[id(o)].data_ptr(),
                              o.mstream.cuda_stream)
        if self.rccl is not None:  # the transfers on the matching stream, behind the pack
            recv = [r.data_ptr() for r in self.recv] if self.rank == 0 else None
            self.rccl.gather([buf.data_ptr()], self.cap_bytes, [recv] if recv else None, 0, o.mstream.cuda_stream)
            o.released = None
            self.transfers += 1
            self.last_set = o
            if self.rank == 0:
                self.last = [buf[:self.cap_bytes] if r == 0 else self.recv[r][:self.cap_bytes]
                             for r in range(self.world)]
            return
        ev = self.packed[id(o)]
        ev.record(o.mstream)
        self.comm.wait_event(ev)
        with torch.cuda.stream(self.comm):
            if self.comm_dev.type == "cpu":  # --rehearse: gloo, staged through the host
                self.comm.synchronize()
                out = gather_fixed(buf.cpu(), self.cap_bytes, dst=0, recv=self.recv)
            else:
                out = gather_fixed(buf, self.cap_bytes, dst=0, recv=self.recv)
        o.released = self.sent[id(o)]
        o.released.record(self.comm)
        self.transfers += 1
        self.last_set = o
        if self.rank == 0:
            self.last = out

    def receive_only(self):
        """Rank 0 on a slot without its own sub-batch (--root-share): the peers' payloads of that
        slot, received into the same buffers, on the matching stream (RCCL) or the comm stream."""
        import torch
        from orb_slam2_2021_amd.parallel import gather_fixed
        assert self.rank == 0
        if self.rccl is not None:
            recv = [r.data_ptr() for r in self.recv]
            self.rccl.gather([0], self.cap_bytes, [recv], 0, self.pipe.mstream.cuda_stream)
        else:
            buf = next(iter(self.bufs.values()))
            with torch.cuda.stream(self.comm):
                gather_fixed(buf.cpu() if self.comm_dev.type == "cpu" else buf, self.cap_bytes, dst=0,
                             recv=self.recv)
        self.transfers += 1


class HostFeed:
    """--feed host: each sub-batch's 2B images go from pinned host memory (the NB distinct input
    batches, page-locked once) into one of R device slots on the pipeline's copy stream, and the
    extraction waits for that copy. After each extraction is enqueued, an event on its stream marks
    the slot consumed (only k_copy0 reads the input images, and the whole extraction is behind the
    event); the copy into slot k mod R for sub-batch k waits for sub-batch k - R's event. R defaults
    to two per extractor handle, so the copies run up to R sub-batches ahead of the extraction and
    the link, not slot reuse, bounds the rate when 2B images take longer to copy than to process
    (round 4 tied the slots to the handles' pyramid events, R = 4: 45.8k stereo frames/s).

    The copies are enqueued `prefetch` sub-batches ahead of the extraction that reads them (at most
    R - 1, so the event a copy waits for is always recorded): when the device queues are full a
    launch blocks the host thread (~55 us each, half of a sub-batch's launches in this mode), and a
    copy enqueued just before its own extraction then starts ~240 us after the previous copy
    finished, leaving the link idle a third of the time (profiles/r6_hostfed_prefetch.txt)."""

    def __init__(self, host, n_img, H, W, dev, copy_stream, slots=0, copy_streams=1, pin="torch", prefetch=-1):
        import torch
        self.pin = pin
        if pin == "register":  # the numpy buffer itself, page-aligned, registered with the runtime
            from orb_slam2_2021_amd import _lib as L
            raw = np.empty(host.nbytes + 4096, np.uint8)
            off = (-raw.ctypes.data) % 4096
            buf = raw[off:off + host.nbytes].view(host.dtype).reshape(host.shape)
            buf[...] = host
            L.check(L.lib().orbfe_host_register(ctypes.c_void_p(buf.ctypes.data), host.nbytes), "host_register")
            self._raw = raw
            self.h = torch.from_numpy(buf)
        else:
            self.h = torch.from_numpy(host).pin_memory()
        # --copy-streams 2: each sub-batch's images as two halves on two copy streams (the second
        # created here, after the pipeline's), joined by an event before the extraction's
        self.cs2 = [torch.cuda.Stream(dev) for _ in range(max(0, copy_streams - 1))]
        self.joined = []
        self.R = 0
        self.slots = None
        self.slots_req = slots
        self.n_img, self.H, self.W, self.dev = n_img, H, W, dev
        self.cs = copy_stream
        self.k = 0        # copies enqueued
        self.taken = 0    # sub-batches handed to the pipeline
        self.prefetch_req = prefetch
        self.prefetch = 0
        self.pending = []
        self.ready = []
        self.consumed = []
        self.bytes_per_subbatch = n_img * H * W

    def take(self, n_of, pipe):
        """The next sub-batch's (slot pointer, ready event); first enqueues the copies of the
        sub-batches up to `prefetch` ahead (n_of(i): the host batch of the i-th sub-batch)."""
        if self.slots is None:
            self._alloc(pipe)
        while self.k <= self.taken + self.prefetch:
            self.pending.append(self.upload(n_of(self.k), pipe))
        self.taken += 1
        return self.pending.pop(0)

    def _alloc(self, pipe):
        import torch
        from orb_slam2_2021_amd.pipeline import new_event
        if self.slots is None:
            self.R = self.slots_req if self.slots_req > 0 else 2 * len(pipe.exts)
            self.prefetch = (self.R - 1) // 2 if self.prefetch_req < 0 else min(self.prefetch_req, self.R - 1)
            self.slots = torch.empty((self.R, self.n_img, self.H, self.W), dtype=torch.uint8, device=self.dev)
            self.ready = [new_event(self.dev.index) for _ in range(self.R)]
            self.consumed = [new_event(self.dev.index) for _ in range(self.R)]
            self.joined = [new_event(self.dev.index) for _ in range(self.R)] if self.cs2 else []

    def upload(self, j, pipe):
        import torch
        if self.slots is None:
            self._alloc(pipe)
        slot = self.k % self.R
        if self.k >= self.R:  # sub-batch k - R's extraction read this slot
            self.consumed[slot].wait(self.cs)
            for c in self.cs2:
                self.consumed[slot].wait(c)
        if self.cs2:
            half = self.n_img // 2
            with torch.cuda.stream(self.cs):
                self.slots[slot][:half].copy_(self.h[j][:half], non_blocking=True)
            with torch.cuda.stream(self.cs2[0]):
                self.slots[slot][half:].copy_(self.h[j][half:], non_blocking=True)
            self.joined[slot].record(self.cs2[0])
            self.joined[slot].wait(self.cs)
        else:
            with torch.cuda.stream(self.cs):
                self.slots[slot].copy_(self.h[j], non_blocking=True)
        self.ready[slot].record(self.cs)
        self.k += 1
        return self.slots[slot].data_ptr(), self.ready[slot]

    def extracted(self, pipe):
        """After pipe.run() of the last uploaded sub-batch: its slot is free once that extraction is."""
        self.consumed[(self.taken - 1) % self.R].record(pipe.last_stream)

    def describe(self, subbatches_per_s):
        gbs = self.bytes_per_subbatch * subbatches_per_s / 1e9
        return {"mode": "host", "h2d_bytes_per_subbatch": self.bytes_per_subbatch, "h2d_GBps": round(gbs, 2),
                "device_slots": self.R, "copies_ahead": self.prefetch,
                "copy_streams": 1 + len(self.cs2),
                "host_pin": self.pin,
                "source_pinned": bool(self.h.is_pinned()),
                "what": "every sub-batch's images H2D from pinned host memory on a copy stream of its own, "
                        "overlapped with the other sub-batches' kernels; outputs stay in HBM"}


class GatherProxy:
    """--gather-proxy N on one GPU: the cost rank 0 pays for C4's ingestion at N GPUs, without the
    peers. Per sub-batch the keypoints + descriptors are packed on the matching stream (as
    Gatherer.pack does); every --gather-every K sub-batches the K packed payloads go through N - 1
    RCCL send / receive pairs each of a world-1 communicator with itself, one group on the matching
    stream (Gatherer's transfer path, orb_slam2_2021_amd.rccl). The self pairs read and write rank
    0's HBM (the send side too, which a real root does not pay): an upper bound on the root's HBM
    and CU cost, no model of the xGMI links."""

    def __init__(self, pipe, n_gpus, dev, every=1):
        import torch
        from orb_slam2_2021_amd.parallel import packed_bytes
        from orb_slam2_2021_amd.rccl import RcclComm, unique_id
        self.pipe, self.n, self.every = pipe, n_gpus, max(1, every)
        self.cap_bytes = packed_bytes(pipe.n_img, pipe.n_img * pipe.cap)
        self.bufs = {id(o): torch.empty(self.cap_bytes, dtype=torch.uint8, device=dev) for o in pipe.sets}
        self.sizes = {id(o): torch.zeros(1, dtype=torch.int64, device=dev) for o in pipe.sets}
        self.recv = [torch.empty(self.cap_bytes, dtype=torch.uint8, device=dev)
                     for _ in range((n_gpus - 1) * self.every)]
        self.rccl = RcclComm(1, 0, unique_id())
        self.pending = []
        self.transfers = 0
        self.last_buf = None

    def pack(self, o):
        from orb_slam2_2021_amd.parallel import pack_keypoints_device
        p, m = self.pipe, o.mstream
        buf = self.bufs[id(o)]
        pack_keypoints_device(p.n_img, o.cnt.data_ptr(), o.kps.data_ptr(), o.desc.data_ptr(), p.cap,
                              buf.data_ptr(), self.cap_bytes, self.sizes[id(o)].data_ptr(), m.cuda_stream)
        self.pending.append(buf.data_ptr())
        self.last_buf = buf.data_ptr()
        if len(self.pending) == self.every:
            # (a set's payload buffer is rewritten only by its next pack, behind this on the stream)
            k = self.n - 1
            recv = [[r.data_ptr() for r in self.recv[j * k:(j + 1) * k]] for j in range(len(self.pending))]
            self.rccl.self_copies(self.pending, self.cap_bytes, recv, m.cuda_stream)
            self.pending = []
        self.transfers += 1

    def receive_only(self):
        """A slot without rank 0's own sub-batch: the N - 1 peer payloads only (self pairs of the
        last packed payload), one group on the matching stream."""
        m = self.pipe.mstream
        src = self.last_buf if self.last_buf is not None else next(iter(self.bufs.values())).data_ptr()
        k = self.n - 1
        self.rccl.self_copies([src], self.cap_bytes, [[r.data_ptr() for r in self.recv[:k]]], m.cuda_stream)
        self.transfers += 1

    def describe(self):
        return {"n_gpus_modelled": self.n, "payloads_per_subbatch": self.n - 1, "bytes_per_payload": self.cap_bytes,
                "received_bytes_per_subbatch": self.cap_bytes * (self.n - 1), "gather_every": self.every,
                "what": "rank 0's ingestion of C4 on one GPU: N-1 RCCL self send / receive pairs of the packed "
                        "worst-case payload per sub-batch on the matching stream, batched every K sub-batches "
                        "into one group; the send side's HBM traffic is counted too (an upper bound)"}


def main():
    args = parse()
    hw_queues = hw_queue_setting(args.hw_queues, max(int(os.environ.get("WORLD_SIZE", "1")), args.gather_proxy))
    if args.feed == "host" and args.hw_queues < 0:
        hw_queues = HW_QUEUES_MULTI_RANK  # the copy stream on a hardware queue of its own
    if hw_queues > 0:  # read once by the HIP runtime at its start (no HIP call before this)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(hw_queues, 32))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    gpu = 0 if (world == 1 or args.rehearse) else local
    torch.cuda.set_device(gpu)
    # the pipeline's busy streams first, before RCCL, torch's stream pool or any handle creates
    # one, so that each opens its own hardware queue (PipelineStreams)
    from orb_slam2_2021_amd.pipeline import PipelineStreams
    n_ext = max(1, args.extractors)
    pstreams = PipelineStreams(gpu, n_ext, match_inline=args.match_inline, side_last=args.inline_side,
                               comm=world > 1, copy=args.feed == "host", high=tuple(args.high_prio.split(",")))
    if world > 1 and args.rehearse:  # every rank on GPU 0, gloo between the processes
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if world > 1:
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", torch.cuda.current_device())
    comm_dev = torch.device("cpu") if args.rehearse else dev  # tensors of the small collectives

    from orb_slam2_2021_amd import ORBextractor, synth_frame
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.parallel import shard_frames
    from orb_slam2_2021_amd.pipeline import build_c3
    from orb_slam2_2021_amd.vocabulary import ORBVocabulary

    B, H, W = args.batch, args.rows, args.cols
    n_img = 2 * B
    NB = max(1, args.input_batches)
    S_sub = max(1, args.batches_per_step)
    # ---- inputs: NB distinct batches of B stereo frames of this rank, resident in HBM ----
    host = make_inputs(args, world, rank)
    d_img = torch.from_numpy(host).to(dev)
    feed = None
    if args.feed == "host":
        feed = HostFeed(host, n_img, H, W, dev, pstreams.copy, slots=args.input_slots, pin=args.host_pin,
                        prefetch=args.copies_ahead,
                        copy_streams=args.copy_streams)
    ext = ORBextractor(args.nfeatures, 1.2, 8, 20, 7, device=dev.index)
    tree = S.Vocabulary.synthetic_orbvoc(levels=args.vocab_levels)
    voc = ORBVocabulary.from_tree(tree, device=dev.index)
    if args.fast_side > 0:
        ext.debug_set_fast_side_levels(args.fast_side)
    if args.blur_mode >= 0:
        ext.debug_set_blur_mode(args.blur_mode)
    if args.inline_side:
        ext.debug_set_inline_side(True)
    exts = [ext]
    n_handles = n_ext * max(1, args.handles_per_stream)
    if n_handles > 1:
        # several handles extract consecutive sub-batches concurrently; their side-stream work
        # shares one high-priority stream (PipelineStreams.side)
        exts += [ORBextractor(args.nfeatures, 1.2, 8, 20, 7, device=dev.index) for _ in range(n_handles - 1)]
        for e in exts:
            if args.inline_side:
                e.debug_set_inline_side(True)
            if args.fast_side > 0:
                e.debug_set_fast_side_levels(args.fast_side)
            # with two handles the other handle's kernels fill the CUs beside DistributeOctTree,
            # and the shared side stream is better left to FAST alone: the blur follows the octree
            # on the handle's own stream (82.0k vs 80.8k stereo frames/s, interleaved runs)
            e.debug_set_blur_mode(args.blur_mode if args.blur_mode >= 0 else 1)
    if args.graphs:
        for e in exts:
            e.set_graphs(True)
    if args.octree_split >= 0:
        for e in exts:
            e.debug_set_octree_split(args.octree_split)
    if args.fast_wpb:
        sw, mw = (int(x) for x in args.fast_wpb.split(","))
        for e in exts:
            e.debug_set_fast_wpb(sw, mw)
    if args.octree_lds:
        hi, lo = (int(x) for x in args.octree_lds.split(","))
        for e in exts:
            e.debug_set_octree_lds(hi, lo)
    if args.octree_threads:
        small, batch = (int(x) for x in args.octree_threads.split(","))
        for e in exts:
            e.debug_set_octree_threads(small, batch)
    if args.fast_side_merge:
        for e in exts:
            e.debug_set_fast_side_merge(True)
    if args.pyramid_tiles:
        t = [int(x) for x in args.pyramid_tiles.split(",")]
        for e in exts:
            e.debug_set_pyramid_tiles((t[0], t[1]), (t[2], t[3]))
    pipe, state = build_c3(exts if len(exts) > 1 else ext, tree, voc, B, H, W, dev, seed=1234 + rank,
                           depth=pipe_depth(args), stereo=args.stereo, levelsup=args.levelsup, streams=pstreams,
                           pairs=args.pairs, stereo_on_match=not args.stereo_on_extract,
                           native=not (args.stage_calls or args.diag_skip_matching))
    if args.diag_skip_matching:  # diagnostic only: the extraction alone (not the metric's workload)
        def extract_only(o, after_match):
            m = o.mstream = pipe.mstream
            m.wait_event(o.extracted)
            o.matched.record(m)
        pipe._match = extract_only
    gather = world > 1 and not args.no_gather
    comm = pstreams.comm
    g = Gatherer(pipe, world, rank, dev, comm_dev, comm) if gather else None
    if args.gather_proxy > 1 and world == 1:
        g = GatherProxy(pipe, args.gather_proxy, dev, every=args.gather_every)
    counter = [0]
    # C4: rank 0 extracts on a share of the slots only (it ingests every peer's payload on all of them)
    n_model = world if isinstance(g, Gatherer) else (args.gather_proxy if isinstance(g, GatherProxy) else 1)
    share = root_share(args.root_share, n_model) if rank == 0 else 1.0
    own = own_slots(S_sub, share)

    def slot(k):
        if own[k]:
            sub_batch()
        else:
            g.receive_only()

    def sub_batch():
        j = counter[0] % NB
        counter[0] += 1
        if feed is not None:  # the images go up from pinned host memory first (copy stream)
            ptr, ready = feed.take(lambda i: i % NB, pipe)
            pipe.run(ptr, after_match=g.pack if g else None, input_ready=ready)
            feed.extracted(pipe)
        else:
            pipe.run(d_img[j].data_ptr(), after_match=g.pack if g else None)

    def barrier():
        if world > 1:
            dist.barrier()

    # all work goes to the pipeline's two non-default streams, ordered by events
    torch.cuda.set_stream(pipe.stream)
    for _ in range(args.warmup):
        for k in range(S_sub):
            slot(k)
    torch.cuda.synchronize()
    # host cost of enqueueing one sub-batch (untimed): two sub-batches right after a synchronize,
    # 24 times, the median -- the device queues stay short, so no launch blocks on a full queue (32
    # back to back, rounds 3-5, could fill them: 88-197 us for the same code)
    host_samples = []
    for _ in range(24):
        torch.cuda.synchronize()
        th0 = time.perf_counter()
        sub_batch()
        sub_batch()
        host_samples.append((time.perf_counter() - th0) / 2)
    host_us = float(np.median(host_samples)) * 1e6
    torch.cuda.synchronize()
    # timed region: every kernel's launches on every n-th group of sub-batches timed by their own
    # dispatch interval (orbfe_ktimer: start / stop events bound to the dispatch, the interval
    # rocprofv3's kernel trace reports) -> device time per sub-batch per kernel, measured under the
    # timed region's own contention; the dominant kernel is the largest
    from orb_slam2_2021_amd import _lib as L
    kt_overhead = L.ktimer_calibrate(dev.index)  # on a private stream, the pipeline idle
    L.ktimer_reset()
    ev_every = max(1, args.event_every)
    timed_events = 0

    def set_events(on):
        if not args.no_kernel_events:
            L.ktimer_select(True if on else None)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for k in range(S_sub):
            ev = (k // len(exts)) % ev_every == 0  # len(exts) consecutive sub-batches: every handle
            if ev:
                set_events(True)
                timed_events += 1
            slot(k)
            if ev:
                set_events(False)
    t_enq = time.perf_counter()  # every launch of the timed region enqueued
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    timed = L.ktimer_read()
    if not timed:  # --no-kernel-events: a short untimed pass with every kernel timed instead
        L.ktimer_select(True)
        for _ in range(args.probe_subbatches):
            sub_batch()
        torch.cuda.synchronize()
        L.ktimer_select(False)
        timed, timed_events = L.ktimer_read(), args.probe_subbatches
    corr = {k: (ms - c * kt_overhead * 1e-3, c) for k, (ms, c) in timed.items()}  # overhead off each launch
    dominant = max(corr, key=lambda k: corr[k][0])
    watch = [dominant] + (["k_fast"] if dominant != "k_fast" and "k_fast" in timed else [])
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # frames of every rank: the peers' S_sub per step each, rank 0's own share
    frames = B * args.steps * ((world - 1) * S_sub + sum(own if rank == 0 else own_slots(S_sub, root_share(
        args.root_share, n_model))))
    value = frames / elapsed
    last = pipe.last
    counts = last.cnt.cpu().numpy()
    cand = pipe.exts[(pipe.counter - 1) % len(pipe.exts)].debug_candidate_total()  # last sub-batch's handle
    nm = last.nm.cpu().numpy()
    geo = ext.geometry(H, W)
    rooflines = []
    for kname in watch:
        r = roofline(timed, kname, geo, counts, cand, n_img, timed_events, pipe, kt_overhead)
        r["measured_in"] = ((f"timed region, every {ev_every}th group of sub-batches ({timed_events} sub-batches)"
                             if not args.no_kernel_events else "an untimed pass after the timed region")
                            + ": start / stop HIP events bound to each launch's dispatch (hipExtLaunchKernelGGL, "
                              "orbfe_ktimer), the kernel's own execution interval as rocprofv3 --kernel-trace reports it")
        r["traffic"], r["traffic_source"] = pmc_traffic(kname, W, H, B, args)
        if r["traffic"] is not None:  # per launch, like `achieved`: the sub-batch figure / its launches
            r["traffic_per_subbatch"] = r["traffic"]
            r["traffic"] = int(r["traffic"] / r["launches_per_subbatch"])
        issue = pmc_issue(kname, r.get("avg_launch_us"), W, H, B, args)
        if issue is not None:
            r["issue"] = issue
        rooflines.append(r)
    roof = rooflines[0]
    roof["dominant_by"] = "device time per sub-batch, every kernel timed on the same sub-batches"
    if len(rooflines) > 1:
        roof["also"] = rooflines[1:]
    algo_frame = pipeline_bytes_per_stereo_frame(geo, counts, B, pipe.n_pairs)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "stereo frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "host_enqueue_ms_per_step": round(1e3 * (t_enq - t0) / args.steps, 4),
        "host_us_per_subbatch_unblocked": round(host_us, 1),
        "launch_graphs": dict(zip(("captures", "replays", "held"), ext.debug_graph_stats())),
        "enqueue": ("one orbfe_c3_run call per sub-batch (include/orbfe_c3.h)" if pipe._c3 is not None
                    else "per-stage library calls from Python (--stage-calls)"),
        **({"diagnostic": "matching skipped: extraction only, not the C3 metric"} if args.diag_skip_matching else {}),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (seeded KITTI-shaped driving sequence, orbfe_synth_sequence_frame, 1 m per frame along z"
                 if args.pairs == "kf" else "synthetic (seeded KITTI-shaped stereo frames, orbfe_synth_frame")
                + "; synthetic ORBvoc-shaped "
                f"vocabulary k=10 L={args.vocab_levels})",
        **({"feed": feed.describe(value / world / B)} if feed is not None else {}),
        "config": {
            "workload": ("host-fed " if feed is not None else "") + "C3: stereo extract + ComputeBoW + "
                        + ("ComputeStereoMatches + " if args.stereo else "")
                        + (f"SearchForTriangulation(KF t, KF t+1) x{pipe.n_pairs}" if args.pairs == "kf"
                           else f"SearchForTriangulation(left, right) x{pipe.n_pairs}")
                        + f", {W}x{H}, batch {B} stereo frames/GPU"
                        + (" + RCCL gather to rank 0 (C4)" if gather else ""),
            "nfeatures": args.nfeatures, "scale_factor": 1.2, "nlevels": 8, "ini_th_fast": 20,
            "min_th_fast": 7, "vocabulary": f"k=10 L={args.vocab_levels} ({tree.n_nodes} nodes), "
                                            f"levelsup {args.levelsup}, TF_IDF / L1",
            "stereo_frames_per_gpu_per_subbatch": B, "subbatches_per_step": S_sub,
            "stereo_frames_per_gpu_per_step": B * S_sub, "distinct_input_batches": NB,
            "extractor_handles": len(exts), "event_every": ev_every,
            "parallelism": f"frame-sharded x{world}",
            "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            "pipeline": (f"{len(exts)} extractor handles on {n_ext} streams (consecutive sub-batches' "
                         f"extractions overlap), {'matching inline' if args.match_inline else ('' if args.stereo_on_extract else 'ComputeStereoMatches + ') + 'vocabulary + matching on its own stream'}, "
                         f"{pipe_depth(args)} output sets" if pipe_depth(args) > 1 else "one sub-batch at a time"),
        },
        **({"gather_proxy": g.describe()} if isinstance(g, GatherProxy) else {}),
        **({"root_share": {"rank0_own_subbatches_per_step": int(sum(own_slots(S_sub, root_share(args.root_share, n_model)))),
                           "subbatches_per_step": S_sub, "share": round(root_share(args.root_share, n_model), 4),
                           "model": f"1 - {ROOT_INGEST_PER_PEER} (N - 1), N = {n_model}" if args.root_share < 0 else "given",
                           "what": "rank 0 runs its own sub-batch on this share of the slots and receives the peers' "
                                   "payloads on every slot (DESIGN.md section 7)"}} if n_model > 1 else {}),
        "roofline": roof,
        "pipeline_hbm": {
            "algorithmic_bytes_per_stereo_frame": int(algo_frame),
            "achieved_GBps": round(algo_frame * value / world / 1e9, 3),
            "frac_of_peak": round(algo_frame * value / world / 1e9 / HBM_PEAK_GBS, 6),
        },
        "kernels_us_per_subbatch": {k: round(1e3 * v[0] / timed_events, 2)
                                    for k, v in sorted(corr.items(), key=lambda kv: -kv[1][0])},
        "kernels_us_per_subbatch_what": ("device execution per sub-batch on the timed region's event sub-batches "
                                         "(dispatch-bound events less the timer's per-dispatch overhead, "
                                         f"{kt_overhead:.2f} us; the contended pipeline; sums exceed the period "
                                         "because kernels overlap)"),
        "keypoints_per_image": round(float(counts.mean()), 1),
        "sft_matches_per_pair": round(float(nm[:pipe.n_pairs].mean()), 1),
        "sft_pairs_per_subbatch": pipe.n_pairs,
        "stereo_matches_per_pair": (round(float((last.ur >= 0).sum().item()) / B, 1) if args.stereo else None),
        "cpu_baseline": None,
    }
    if isinstance(g, Gatherer) and rank == 0:
        from orb_slam2_2021_amd.parallel import packed_size
        used = [packed_size(v) for v in g.last]
        out["gather"] = {"bytes_sent_per_rank_per_subbatch": g.cap_bytes,
                         "used_bytes_last_subbatch": used,
                         "bytes_received_per_subbatch": g.cap_bytes * (world - 1),
                         "what": "packed keypoints + descriptors of ranks 1..N-1 to rank 0, point-to-point, "
                                 "fixed worst-case byte count (no size exchange, no host sync per sub-batch)"}
    if isinstance(g, Gatherer) and args.dump_gather:
        dump_gather(args.dump_gather, g, pipe, rank, world)
    # ---- parity of the last timed sub-batch (every rank checks its own) ----
    if not args.no_parity:
        from oracle.c3_check import check_c3
        from oracle.orbref import RefVocabulary
        ref_voc = RefVocabulary.from_table(tree.k, tree.levels, tree.scoring, tree.weighting, tree.parent,
                                           tree.is_leaf, tree.descriptors, tree.weights)
        j = (counter[0] - 1) % NB
        r = check_c3(host[j], pipe.to_host(last), ref_voc, state["u_right"], state["mp_state"], state["scale"],
                     state["sigma2"], state["cam"], state["F12"], state["epipole"], levelsup=args.levelsup,
                     stereo=args.stereo, mb=state["mb"], pairs=args.pairs)
        ok = bool(r["all"])
        if world > 1:
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=comm_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = bool(t.item())
        out["parity_bit_exact"] = ok
        out["parity"] = {k: v for k, v in r.items() if k != "all"}
        out["parity"]["what"] = ("last timed sub-batch of every rank vs the oracle chain (extract, "
                                 "vocabulary transform, SearchForTriangulation): keypoints, descriptors, "
                                 "BowVector, FeatureVector, match12")
    if args.rehearse:
        out["rehearsal"] = "N ranks on one GPU over gloo, host-staged: not a measurement"
    if world > 1 and not args.no_legs:
        out["legs"] = {"c5_search_local_points": c5_leg(args, world, rank, comm_dev)}
    if rank == 0 and world == 1:
        # the host-buffer legs use the first handle with the one-handle blur placement; its side
        # work stays on the pipeline's side stream, created before the handles' own streams
        # (measured: 20.7k / 19.6k stereo frames/s on the handle's own side stream, 22.1-22.9k
        # on the pipeline's)
        torch.cuda.synchronize()
        ext.debug_set_blur_mode(args.blur_mode if args.blur_mode >= 0 else 0)
        out["host_boundary"] = host_boundary_rate(ext, host[0], others=exts[1:])
        if not args.no_legs:
            out["c2_latency"] = c2_latency(args, host[0][0], host[0][B])
            out["legs"] = {"c3_host_fed": host_fed_leg(args),
                           "tracking_sequence": tracking_leg(args),
                           "c5_search_local_points": c5_leg(args, 1, 0, dev),
                           "keyframe_searches": keyframe_leg(args),
                           "compute_stereo_matches": stereo_leg(args, ext, d_img[0], host[0], B, H, W,
                                                                pipe.cap, state["cam"]["bf"], state["mb"]),
                           "vocabulary_transform": vocab_leg(args, voc, tree, pipe),
                           "c3_other_pairing": pairing_leg(args, exts, tree, voc, d_img, pstreams, dev)}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(host[0], B, H, W, args, tree, state)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        if isinstance(g, Gatherer) and g.rccl is not None:
            torch.cuda.synchronize()
            g.rccl.close()
        dist.destroy_process_group()


def host_fed_leg(args, steps=3, subbatches=256):
    """The C3 step fed from host memory (bench.py --feed host as a child process, so that its copy
    stream gets a hardware queue of its own): the reference's operator() takes host images
    (ORBextractor.cc:1041-1048, two per stereo Frame, Frame.cc:113-116), so this is the rate a
    host-resident image stream gets; the headline keeps the inputs in HBM."""
    cmd = [sys.executable, os.path.abspath(__file__), "--feed", "host", "--steps", str(steps), "--warmup", "1",
           "--batches-per-step", str(subbatches), "--no-legs", "--no-cpu", "--event-every", "1000000"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return "timeout"
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return f"rc {r.returncode}: {r.stderr[-400:]}"
    d = json.loads(lines[-1])
    return {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps": d["steps"],
            "subbatches_per_step": d["config"]["subbatches_per_step"], "feed": d.get("feed"),
            "parity_bit_exact": d.get("parity_bit_exact"), "hw_queues": d["config"]["hw_queues"],
            "link_bound_stereo_frames_per_s_at_53GBps": round(53e9 / d["feed"]["h2d_bytes_per_subbatch"] * args.batch, 1),
            "what": "bench.py --feed host (child process): C3 with every sub-batch's images copied H2D from pinned "
                    "host memory, overlapped with the kernels; not the metric (inputs resident in HBM)"}


def dump_gather(d, g, pipe, rank, world):
    """--dump-gather: rank r writes its last gathered sub-batch as extracted (r_own.npz); rank 0
    writes every rank's payload as received (r_gathered.bin). tests/test_gpu_gather.py compares
    them byte for byte."""
    import torch
    torch.cuda.synchronize()
    os.makedirs(d, exist_ok=True)
    h = pipe.to_host(g.last_set)
    np.savez(os.path.join(d, f"{rank}_own.npz"),
             kps=np.concatenate(h["keypoints"]).view(np.uint8) if h["keypoints"] else np.zeros(0, np.uint8),
             desc=np.concatenate(h["descriptors"]).reshape(-1), counts=np.array([len(k) for k in h["keypoints"]]))
    if rank == 0:
        for r, v in enumerate(g.last):
            v.cpu().numpy().tofile(os.path.join(d, f"{r}_gathered.bin"))


def pipe_depth(args):
    """Output sets in flight: --pipeline, or 2 per extractor handle (sub-batch i's set is reused
    by i + depth, whose handle then finished i + depth - n_ext's extraction long before)."""
    return args.pipeline if args.pipeline > 0 else 2 * max(1, args.extractors) * max(1, args.handles_per_stream)


def level_pixels(geo):
    return [int(w) * int(h) for w, h in geo[:, :2]]


def roofline(kt, dom, geo, counts, n_cand, n_img, subbatches, pipe, overhead_us=0.0):
    """Roofline of kernel `dom`: ALGORITHMIC bytes per sub-batch / its device time per sub-batch
    (kt: {kernel: (total ms, launches)} over `subbatches` sub-batches; a kernel may run as several
    launches per sub-batch, e.g. k_resize_win once per level and k_fast as levels 0-2 beside the
    resize chain + levels 3..7; per launch = per sub-batch / launches). Algorithmic bytes per
    sub-batch of n_img images (input read once, output written once):
      k_copy0          2 px_0 per image
      k_resize_win     sum_l>=1 (px_{l-1} + px_l) per image
      k_pyramid        2 px_0 + sum_l>=1 px_l per image
      k_fast           sum_l px_l per image + 4 B per cell count + 4 B per FAST candidate
      k_octree         2 x 4 B per candidate (gather + partition) + 4 B per survivor
      k_blur           2 sum_l px_l per image
      k_describe       4 B in + 60 B out per keypoint (the 749 + 512 window bytes a keypoint
                       gathers overlap between keypoints and come from L2: not counted)
      k_stereo_rows    (28 + 16) B per right keypoint
      k_stereo_match   (28 + 32) B per left keypoint + (32 + 16) B per right keypoint + 12 B out per
                       left keypoint (the SAD windows come from L2: not counted)
      k_stereo_median  8 B per left keypoint
      k_vocab_descend  32 B in + 6 x 48 B child records + 8 B out per KeyFrame descriptor
      k_vocab          8 B in + 24 B out (FeatureVector + BowVector) per KeyFrame descriptor
      k_sft_nodes      per pair (N1 + N2)(32 + 28 + 4) B + 4 N1 out
      k_sft_finish     per pair 4 N1"""
    px = level_pixels(geo)
    ncells = int(geo[:, 2].sum())
    nkp = int(counts.sum())
    B = n_img // 2
    n_left, n_right = int(counts[:B].sum()), int(counts[B:].sum())
    n_voc = int(counts[:pipe.n_vocab].sum())
    per_sub = {
        "k_copy0": n_img * 2 * px[0],
        "k_resize_win": n_img * sum(px[l - 1] + px[l] for l in range(1, len(px))),
        "k_pyramid": n_img * (2 * px[0] + sum(px[1:])),
        "k_fast": n_img * (sum(px) + 4 * ncells) + 4 * n_cand,
        "k_octree": 8 * n_cand + 4 * nkp,
        "k_blur": n_img * 2 * sum(px),
        "k_describe": 64 * nkp,
        "k_stereo_rows": 44 * n_right,
        "k_stereo_match": 72 * n_left + 48 * n_right,
        "k_stereo_median": 8 * n_left,
        "k_vocab_descend": (32 + 6 * 48 + 8) * n_voc,
        "k_vocab": 32 * n_voc,
        "k_sft_nodes": sum(64 * int(counts[a] + counts[b]) + 4 * int(counts[a]) for a, b in pipe.pair_idx),
        "k_sft_finish": sum(4 * int(counts[a]) for a, _ in pipe.pair_idx),
    }
    total_ms, launches = kt[dom]
    per_launch = max(round(launches / max(subbatches, 1)), 1)  # launches per sub-batch
    raw_s = total_ms / 1e3 / max(subbatches, 1)
    # the timer's own per-dispatch overhead (orbfe_ktimer_calibrate) off every launch
    sub_s = max(raw_s - launches * overhead_us * 1e-6 / max(subbatches, 1), 1e-9)
    algo = per_sub.get(dom)
    out = {"kernel": dom, "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
           "traffic": None, "kernel_us_per_subbatch": round(sub_s * 1e6, 2),
           "avg_launch_us": round(sub_s * 1e6 / per_launch, 2), "launches_per_subbatch": per_launch,
           "avg_launch_us_events": round(raw_s * 1e6 / per_launch, 2), "timer_overhead_us": round(overhead_us, 2)}
    if algo is not None:
        achieved = algo / sub_s / 1e9
        out.update({"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 6),
                    "algorithmic_bytes_per_subbatch": int(algo), "algorithmic_bytes_per_launch": int(algo / per_launch)})
    return out


def pmc_workload(W, H, B, args):
    return {"cols": W, "rows": H, "batch": B, "pairs": args.pairs, "stereo": bool(args.stereo)}


def pmc_traffic(kernel, W, H, B, args):
    """HBM bytes per sub-batch of `kernel` from the committed rocprofv3 PMC summary of this workload
    (profiles/pmc_traffic.json, written by profiles/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of bench.py; FETCH_SIZE doubled per MI355X_MICROARCH.md), or None when no
    summary for this kernel and workload is committed."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None, None
    if doc.get("workload") != pmc_workload(W, H, B, args):
        return None, None
    k = doc.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return int(k["traffic_bytes_per_step"]), doc.get("source")


SIMDS = 1024             # 256 CUs x 4 SIMD-32 (MI355X_MICROARCH.md)
ISSUE_CLOCK_GHZ = 2.4    # max engine clock
VALU_CYCLES_WAVE64 = 2   # a wave64 VALU instruction on a SIMD-32 with two or more waves resident


def pmc_issue(kernel, avg_launch_us, W, H, B, args):
    """The VALU-issue roof of `kernel` beside its HBM roof: SQ_INSTS_VALU per launch (committed
    rocprofv3 PMC summary of this workload, profiles/pmc_waits.json from profiles/pmc_waits.py)
    x 2 cycles / (1,024 SIMDs x 2.4 GHz x the launch time this run measured), with the PMC run's
    wave-time split (issuing / ready but not issued / parked on waitcnt or barriers) and resident
    waves per SIMD. None when no summary for this kernel and workload is committed."""
    path = os.path.join(ROOT, "profiles", "pmc_waits.json")
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    if doc.get("workload") != pmc_workload(W, H, B, args) or not avg_launch_us:
        return None
    k = doc.get("kernels", {}).get(kernel)
    if not k:
        return None
    issue_us = k["insts_valu_per_launch"] * VALU_CYCLES_WAVE64 / (SIMDS * ISSUE_CLOCK_GHZ * 1e3)
    return {"bound": "valu_issue", "valu_insts_per_launch": int(k["insts_valu_per_launch"]),
            "issue_us_per_launch": round(issue_us, 2), "frac": round(issue_us / avg_launch_us, 4),
            "wave_split": {"issuing": round(k["active"], 3), "ready_not_issued": round(k["wait_inst"], 3),
                           "parked": round(k["wait_any"], 3)},
            "waves_per_simd": round(k["waves_per_simd"], 2),
            "formula": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x avg_launch_us)",
            "source": doc.get("source")}


def pipeline_bytes_per_stereo_frame(geo, counts, B, n_pairs):
    """per image sum_l px (read once) + sum_l>=1 px (write) + 60 B per keypoint;
    SearchForTriangulation per pair 2 N (32 + 28 + 4) + N/4 + 8 N, n_pairs pairs per B frames."""
    px = level_pixels(geo)
    n_per_img = float(counts.mean())
    extract = sum(px) + sum(px[1:]) + 60 * n_per_img
    sft = 2 * n_per_img * 64 + 2 * n_per_img / 8 + 4 * 2 * n_per_img
    return 2 * extract + sft * n_pairs / B


def percentiles(xs):
    a = np.sort(np.asarray(xs)) * 1e3
    return {"p50_ms": round(float(np.percentile(a, 50)), 4), "p99_ms": round(float(np.percentile(a, 99)), 4),
            "min_ms": round(float(a[0]), 4), "n": len(a)}


def c2_latency(args, left, right, reps=200):
    """BASELINE config C2: one 1241x376 image through the drop-in orbfe_extract (host buffers in
    and out: H2D, kernels, D2H, what ORBextractor::operator() costs a caller), and the stereo
    Frame's pattern (Frame.cc:113-116): two extractor handles on two threads, one image each.
    Wall-clock latency per call from preallocated host buffers; parity vs the oracle for one image."""
    from ctypes import byref, c_int, c_size_t
    from orb_slam2_2021_amd import ORBextractor
    from orb_slam2_2021_amd import _lib as L
    lib = L.lib()
    rows, cols = left.shape
    exts = [ORBextractor(args.nfeatures, 1.2, 8, 20, 7) for _ in range(2)]
    cap = exts[0].max_keypoints(rows, cols)
    bufs = [(np.zeros(cap, L.KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8), c_int()) for _ in range(2)]
    imgs = [np.ascontiguousarray(left), np.ascontiguousarray(right)]

    def call(s):
        k, d, n = bufs[s]
        L.check(lib.orbfe_extract(exts[s]._h, L.ptr(imgs[s]), rows, cols, c_size_t(cols), L.ptr(k), cap,
                                  L.ptr(d), byref(n)), "orbfe_extract")

    for _ in range(10):
        call(0)
        call(1)
    single = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call(0)
        single.append(time.perf_counter() - t0)
    # the same call replayed from a captured hipGraph (orbfe_extractor_set_graphs(1))
    exts[0].set_graphs(True)
    for _ in range(10):
        call(0)
    graphed = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call(0)
        graphed.append(time.perf_counter() - t0)
    exts[0].set_graphs(False)
    pair = []
    go = [threading.Event(), threading.Event()]
    done = [threading.Event(), threading.Event()]
    stop = [False]

    def worker(s):
        while True:
            go[s].wait()
            go[s].clear()
            if stop[0]:
                return
            call(s)
            done[s].set()

    th = [threading.Thread(target=worker, args=(s,), daemon=True) for s in range(2)]
    for t in th:
        t.start()
    for _ in range(reps + 10):
        t0 = time.perf_counter()
        for s in range(2):
            go[s].set()
        for s in range(2):
            done[s].wait()
            done[s].clear()
        pair.append(time.perf_counter() - t0)
    stop[0] = True
    for s in range(2):
        go[s].set()
    for t in th:
        t.join()
    # the MI355X way to serve the stereo Frame: both images in one orbfe_extract_batch call (one
    # launch sequence) on one handle
    from ctypes import c_void_p
    kb = np.empty(2 * cap, L.KEYPOINT_DTYPE)
    db = np.empty((2 * cap, 32), np.uint8)
    cb = np.zeros(2, np.int32)
    arr = (c_void_p * 2)(imgs[0].ctypes.data, imgs[1].ctypes.data)

    def call_pair():
        L.check(lib.orbfe_extract_batch(exts[0]._h, 2, ctypes.cast(arr, c_void_p), rows, cols, c_size_t(cols),
                                        L.ptr(kb), L.ptr(db), cap, L.ptr(cb)), "orbfe_extract_batch")

    for _ in range(10):
        call_pair()
    one_call = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call_pair()
        one_call.append(time.perf_counter() - t0)
    out = {"single_image": percentiles(single), "single_image_graph_replay": percentiles(graphed),
           "stereo_two_threads": percentiles(pair[10:]),
           "stereo_pair_one_call": percentiles(one_call), "adapter": adapter_latency(),
           "what": "orbfe_extract wall-clock per call (host buffers in and out), 1241x376, 1 GPU; stereo_two_threads "
                   "= two handles on two threads as Frame.cc:113-116; stereo_pair_one_call = both images in one "
                   "orbfe_extract_batch call on one handle; single_image_graph_replay = the same call with the launch "
                   "sequence replayed from a captured hipGraph (orbfe_extractor_set_graphs, off by default)"}
    if not args.no_cpu:
        from oracle.orbref import RefExtractor
        k, d, n = bufs[0]
        kr, dr = RefExtractor(args.nfeatures, 1.2, 8, 20, 7)(imgs[0])
        m = n.value
        out["parity_bit_exact"] = bool(m == len(kr) and all(np.array_equal(k[:m][f], kr[f]) for f in
                                                            ("x", "y", "size", "response", "octave"))
                                       and np.max(np.abs(k[:m]["angle"] - kr["angle"])) <= 1e-5
                                       and np.array_equal(d[:m], dr))
    return out


def adapter_latency(iters=200):
    """The reference-side drop-in adapters (adapter/ORBextractor_gpu.cc + adapter/Frame_gpu.cc, built
    over tests/cpp/cvstub by __graft_entry__.build()) as the reference calls them: ORBextractor::
    operator() on one image with its cv::Mat outputs and mvImagePyramid, and the stereo Frame
    constructor's two ExtractORB threads + ComputeStereoMatches (Frame.cc:113-125). Two builds:
    mvImagePyramid prefetched to the host (the CPU ComputeStereoMatches' input) and
    ORBFE_ADAPTER_GPU_STEREO=1 (no pyramid copy). Child processes (tests/cpp/adapter_latency.cpp)."""
    out = {}
    for name in ("adapter_latency", "adapter_latency_gpustereo"):
        exe = os.path.join(ROOT, "tests", "cpp", "build", name)
        if not os.path.exists(exe):
            out[name] = "not built"
            continue
        try:
            r = subprocess.run([exe, str(iters)], capture_output=True, text=True, timeout=120)
        except subprocess.TimeoutExpired:
            out[name] = "timeout"
            continue
        rec = [l for l in r.stdout.splitlines() if l.startswith("ADAPTER ")]
        out[name] = json.loads(rec[-1][len("ADAPTER "):]) if r.returncode == 0 and rec else f"rc {r.returncode}"
    return out


def c5_scene(nfeatures, world, rank, dev, m_points=50000, frames_per_rank=16):
    """BASELINE config C5's inputs: 640x480 frames of this rank (frame sharding) with their poses,
    and the 50k-MapPoint local map (seed 0x50C0DE) built identically on every rank,
    replicated from rank 0 over the process group when N > 1."""
    from orb_slam2_2021_amd import ORBextractor, synth_frame
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import MapPointGeometry
    from orb_slam2_2021_amd.parallel import broadcast_arrays, shard_frames
    import torch
    gpu = torch.cuda.current_device()  # this rank's GPU (dev may be the host in --rehearse)
    ext = ORBextractor(nfeatures, 1.2, 8, 12, 7, device=gpu)  # arducam.yaml:126-127
    sc, s2 = ext.GetScaleFactors(), ext.GetScaleSigmaSquares()
    k0, d0 = ext(synth_frame(7, 480, 640))
    rng = np.random.default_rng(0x50C0DE)
    F0 = S.make_frame(k0, d0, sc, s2, 480, 640, S.ARDUCAM_CAM, rng, mp_frac=0.0, tcw=S.pose(tx=0.1, yaw=0.02))
    G = S.make_local_map(F0, m_points, rng)  # identical on every rank (same seed)
    fields = ("flags", "world_pos", "normal", "min_distance", "max_distance", "descriptors")
    if world > 1:  # the replicated SoA: rank 0's map broadcast to every rank
        arrs = {f: np.ascontiguousarray(getattr(G, f)) for f in fields}
        got = broadcast_arrays(arrs, dev, src=0)  # dev: the rank's GPU (host in --rehearse)
        G = MapPointGeometry(**{f: got[f].cpu().numpy().view(arrs[f].dtype).reshape(arrs[f].shape)
                                for f in fields})
    n_total = world * frames_per_rank
    mine = shard_frames(n_total, world, rank)
    imgs = [synth_frame(100 + i, 480, 640) for i in mine]
    poses = [S.pose(tx=0.1 + 0.002 * (i % 8), yaw=0.02 + 0.001 * (i % 5)) for i in mine]
    return ext, F0, G, imgs, poses, n_total


def c5_frame(ext, img, tcw):
    from orb_slam2_2021_amd import synthetic as S
    k, d = ext(img)
    return S.Frame(keys_un=k, descriptors=d if d is not None else np.zeros((0, 32), np.uint8),
                   u_right=np.full(len(k), -1.0, np.float32), mp_state=np.zeros(len(k), np.uint8),
                   scale_factors=ext.GetScaleFactors(), level_sigma2=ext.GetScaleSigmaSquares(), min_x=0.0,
                   max_x=640.0, min_y=0.0, max_y=480.0, tcw=tcw, **S.ARDUCAM_CAM)


def c5_leg(args, world, rank, dev, m_points=50000, frames_per_rank=192):
    """BASELINE config C5: a 640x480 stream through Tracking::SearchLocalPoints' hot part --
    Frame::isInFrustum(pMP, 0.5) for every MapPoint of the local map, then
    ORBmatcher(0.8).SearchByProjection(F, vpLocalMapPoints, th=3) (Tracking.cc:1186-1213) -- with
    frames sharded over the ranks and the 50k-MapPoint local map replicated (built on rank 0,
    broadcast over RCCL when N > 1). Per frame: extraction (ORBextractor 12/7, arducam.yaml) and
    orbfe_search_local_points (host-buffer call: frame + map uploaded, PCIe included). frames/s =
    all ranks' frames / max-over-ranks wall time. Then the device part alone: HIP events around
    k_frustum .. the last SearchByProjection kernel of each search (orbfe_matcher_set_profiling),
    and its roofline against SURVEY 8(d)'s bytes: isInFrustum 49 B in + 21 B out per MapPoint,
    SearchByProjection M (32 + 20) + N (32 + 16 + 4) + 3072 x 8 per frame (2.73 MB at 50k), the
    PMC traffic of the same kernels from profiles/pmc_traffic_c5.json. Rank 0 checks its first
    frame bit-exact against the oracle."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from orb_slam2_2021_amd import ORBextractor, ORBmatcher
    from orb_slam2_2021_amd.frames import DeviceMapPointGeometry, log_scale_factor
    ext, F0, G, imgs, poses, n_total = c5_scene(args.nfeatures, world, rank, dev, m_points, frames_per_rank)
    gpu = torch.cuda.current_device()
    m = ORBmatcher(0.8, True, device=gpu)  # Tracking.cc:1206
    # several Tracking-like callers per GPU, each with its own extractor + matcher handle (own
    # streams) on its own thread: one caller's uploads, extraction and claim rounds overlap the
    # others' (the frames are independent; ctypes releases the GIL inside the library calls)
    workers = max(1, args.c5_workers)
    handles = [(ext, m)] + [(ORBextractor(args.nfeatures, 1.2, 8, 12, 7, device=gpu), ORBmatcher(0.8, True, device=gpu))
                            for _ in range(workers - 1)]
    # the replicated local map resident in HBM, uploaded once per rank (after the broadcast when
    # N > 1): the matcher copies it on the device instead of staging 3.3 MB through the host per
    # search; the one-caller rate below passes host arrays, the drop-in call as Tracking makes it
    Gd = DeviceMapPointGeometry(G, device=torch.device("cuda", gpu))
    for e, mm in handles:
        e(imgs[0])
        mm.SearchLocalPoints(F0, Gd, 3.0)

    def run(w, nw, geom):
        e, mm = handles[w]
        res = []
        for i in range(w, len(imgs), nw):
            F = c5_frame(e, imgs[i], poses[i])
            nm, best, nv, _ = mm.SearchLocalPoints(F, geom, 3.0)
            res.append((i, F, nm, best, nv))
        return res

    def timed(nw, geom):
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=nw) as pool:
            res = sorted((r for part in pool.map(lambda w: run(w, nw, geom), range(nw)) for r in part),
                         key=lambda r: r[0])
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dt = float(t.item())
        return dt, res

    dt1, res1 = timed(1, G)  # one caller with host arrays: Tracking's own frame-after-frame call
    dt, res = timed(workers, Gd)
    same = all(a[2] == b[2] and a[4] == b[4] and np.array_equal(a[3], b[3]) for a, b in zip(res1, res))
    nm_total = sum(r[2] for r in res)
    frames = [r[1] for r in res]
    first = res[0][1:]
    # the device part alone (no extraction, no PCIe)
    m.set_profiling(True)
    dev_ms, rounds = [], []
    for _ in range(1):
        for F in frames:
            m.SearchLocalPoints(F, Gd, 3.0)
            dev_ms.append(m.last_device_ms())
            rounds.append(m.last_stats()[0])
    m.set_profiling(False)
    M = len(G.flags)
    N = float(np.mean([F.N for F in frames]))
    algo = M * (49 + 21) + M * (32 + 20) + N * (32 + 16 + 4) + 3072 * 8
    us = 1e3 * float(np.median(dev_ms))
    achieved = algo / (us * 1e-6) / 1e9
    traffic = c5_pmc_traffic(M)
    out = {"frames_per_s": round(n_total / dt, 1), "ms_per_frame_per_rank": round(1e3 * dt / len(imgs), 3),
           "callers_per_rank": workers, "frames_per_s_one_caller_host_map": round(n_total / dt1, 1),
           "resident_map_equals_host_map": bool(same),
           "frames": n_total, "ranks": world, "map_points": M,
           "matches_per_frame_rank0": round(nm_total / len(imgs), 1),
           "device_us_per_search": round(us, 2),
           "claim_rounds_per_search": round(float(np.mean(rounds)), 1),
           "roofline": {"kernel": "k_frustum + k_sbp_* (isInFrustum + SearchByProjection, one frame)",
                        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                        "algorithmic_bytes_per_frame": int(algo),
                        "measured_in": "HIP events around the device part of each search (orbfe_matcher_set_profiling)"},
           "what": "640x480 frames sharded over ranks, local map replicated (broadcast from rank 0 when N > 1); "
                   "per frame ORBextractor + orbfe_search_local_points (host buffers, PCIe included), "
                   f"the local map resident in HBM (uploaded once per rank), {workers} callers per rank on "
                   "their own handles and threads; frames_per_s_one_caller_host_map: one caller frame after "
                   "frame passing the map as host arrays (staged per search)"}
    if rank == 0 and not args.no_cpu:
        from oracle import orbref
        F, nm, best, nv = first
        t0 = time.perf_counter()
        nr, br, nvr, _ = orbref.search_local_points(F, G, log_scale_factor(1.2), 3.0, 0.8, kind="native")
        out["cpu_oracle_ms_per_search"] = round(1e3 * (time.perf_counter() - t0), 3)
        out["cpu_bit_exact"] = bool(nr == nm and nvr == nv and np.array_equal(br, best))
    return out


def tracking_leg(args, n_frames=24, n_last=1500, m_local=8000, cpu_frames=4):
    """Tracking's per-frame device sequence on one GPU (Tracking.cc:210,
    887-911, 1164-1216), frame after frame as Tracking calls it through the drop-in C ABI:
      1. the stereo Frame (Frame.cc:113-125): orbfe_stereo_frame = ORBextractor on left + right,
         then ComputeStereoMatches;
      2. TrackWithMotionModel's matching: SearchByProjection(CurrentFrame, LastFrame, th = 7,
         bMono = false), again at 2 th below 20 matches (ORBmatcher(0.9, true));
      3. SearchLocalPoints: isInFrustum(pMP, 0.5) for the local map, then
         ORBmatcher(0.8).SearchByProjection(F, vpLocalMapPoints, th = 1) with the motion model's
         matches holding their keypoints.
    Frames: the bench's KITTI-shaped driving sequence (1241x376, 1 m per frame). The last frame's
    MapPoints and the local map are synthetic (S.make_lastframe / S.make_local_map around each
    frame's keypoints), built before the timed pass. Host buffers in and out (PCIe included):
    latency per frame = what Tracking waits. Device part: every kernel of the sequence timed by its
    dispatch (orbfe_ktimer), summed per frame. CPU: the oracle (-O3 -march=native, one thread)
    runs the same sequence on the first `cpu_frames` frames, which must match bit for bit."""
    from orb_slam2_2021_amd import ORBextractor, ORBmatcher, synth_sequence_frame
    from orb_slam2_2021_amd import _lib as L
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import log_scale_factor
    H, W = 376, 1241
    cam = S.KITTI_CAM
    mb = cam["bf"] / cam["fx"]
    frames = [synth_sequence_frame(SEQ_SEED, 200 + t, H, W, right=True) for t in range(n_frames)]
    ext = ORBextractor(args.nfeatures, 1.2, 8, 20, 7)
    mm = ORBmatcher(0.9, True)   # Tracking.cc:889
    ml = ORBmatcher(0.8, True)   # Tracking.cc:1207
    scale, sigma2 = ext.GetScaleFactors(), ext.GetScaleSigmaSquares()

    def frame_of(kl, dl, ur, t):
        return S.Frame(keys_un=kl, descriptors=dl if dl is not None else np.zeros((0, 32), np.uint8), u_right=ur,
                       mp_state=np.zeros(len(kl), np.uint8), scale_factors=scale, level_sigma2=sigma2,
                       min_x=0.0, max_x=float(W), min_y=0.0, max_y=float(H), tcw=S.pose(tz=-float(200 + t)), **cam)

    # the synthetic map state around each frame (untimed)
    scene = []
    for t, (l, r) in enumerate(frames):
        kl, dl, _, _, ur, _ = ext.stereo_frame(l, r, cam["bf"], mb)
        F = frame_of(kl, dl, ur, t)
        rng = np.random.default_rng(0x7AC0 + t)
        scene.append((S.make_lastframe(F, n_last, rng, None), S.make_local_map(F, m_local, rng)))

    def run_frame(t):
        l, r = frames[t]
        kl, dl, kr, dr, ur, _ = ext.stereo_frame(l, r, cam["bf"], mb)
        F = frame_of(kl, dl, ur, t)
        last, local = scene[t]
        nm1, best1, th = mm.SearchByProjectionMotionModel(F, last, 7.0, False)
        F.mp_state[best1[best1 >= 0]] = L.ORBFE_MP_OBSERVED  # CurrentFrame.mvpMapPoints[bestIdx2] = pMP
        nm2, best2, nv, _ = ml.SearchLocalPoints(F, local, 1.0)
        return (kl, dl, kr, dr, ur, nm1, best1, th, nm2, best2, nv)

    for t in range(3):
        run_frame(t)
    lat, outs = [], []
    for t in range(n_frames):
        t0 = time.perf_counter()
        outs.append(run_frame(t))
        lat.append(time.perf_counter() - t0)
    L.ktimer_reset()
    L.ktimer_select(True)
    for t in range(n_frames):
        run_frame(t)
    L.ktimer_select(False)
    kt = L.ktimer_read()
    dev_us = {k: round(1e3 * v[0] / n_frames, 2) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])}
    dev_total = sum(v[0] for v in kt.values()) / n_frames * 1e3  # us per frame, kernels back to back
    # algorithmic bytes per frame (every input read once, every output written once)
    geo = ext.geometry(H, W)
    px = level_pixels(geo)
    nl_ = float(np.mean([len(o[0]) for o in outs]))
    nr_ = float(np.mean([len(o[2]) for o in outs]))
    extract = 2 * (sum(px) + sum(px[1:])) + 60 * (nl_ + nr_)
    stereo = 72 * nl_ + 48 * nr_ + 44 * nr_ + 8 * nl_
    sbp_last = n_last * (12 + 32 + 4 + 4 + 1 + 4) + nl_ * (28 + 32 + 4 + 1) + 3072 * 8
    frustum = m_local * (49 + 21)
    sbp_local = m_local * (32 + 20) + nl_ * (32 + 16 + 4) + 3072 * 8
    algo = extract + stereo + sbp_last + frustum + sbp_local
    achieved = algo / (dev_total * 1e-6) / 1e9
    out = {"frames": n_frames, "latency_ms": percentiles(lat), "frames_per_s_one_caller": round(n_frames / sum(lat), 1),
           "device_us_per_frame": round(dev_total, 2), "device_us_per_frame_by_kernel": dev_us,
           "keypoints_left": round(nl_, 1), "last_frame_mappoints": n_last, "local_map_mappoints": m_local,
           "motion_model_matches": round(float(np.mean([o[5] for o in outs])), 1),
           "motion_model_retries": int(sum(o[7] != 7.0 for o in outs)),
           "local_map_in_view": round(float(np.mean([o[10] for o in outs])), 1),
           "local_map_matches": round(float(np.mean([o[8] for o in outs])), 1),
           "roofline": {"kernel": "the whole per-frame sequence (stereo Frame, SearchByProjection(F, LastFrame), "
                                  "isInFrustum + SearchByProjection(F, local map))",
                        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                        "algorithmic_bytes_per_frame": int(algo),
                        "measured_in": "every kernel of the sequence timed by its dispatch (orbfe_ktimer), summed "
                                       "per frame"},
           "what": "Tracking's per-frame device sequence through the host-buffer C ABI, one caller, frame after frame "
                   "(1241x376 driving sequence; synthetic last-frame MapPoints and local map)"}
    if not args.no_cpu:
        from oracle import orbref

        def oracle_frame(t, kind, rx):
            l, r = frames[t]
            kl, dl = rx[0](l)
            kr, dr = rx[1](r)
            ur, _ = orbref.compute_stereo_matches(kl, dl, kr, dr, [rx[0].level(i) for i in range(8)],
                                                  [rx[1].level(i) for i in range(8)], scale, inv, mb, cam["bf"],
                                                  kind=kind)
            F = frame_of(kl, dl, ur, t)
            last, local = scene[t]
            nm1, best1, th = orbref.motion_model_search(F, last, 7.0, False, True, kind=kind)
            F.mp_state[best1[best1 >= 0]] = L.ORBFE_MP_OBSERVED
            nm2, best2, nv, _ = orbref.search_local_points(F, local, log_scale_factor(1.2), 1.0, 0.8, kind=kind)
            return (kl, dl, kr, dr, ur, nm1, best1, th, nm2, best2, nv)

        n = min(cpu_frames, n_frames)
        # timing: the oracle built with the reference's flags (-O3 -march=native)
        rx = [orbref.RefExtractor(args.nfeatures, 1.2, 8, 20, 7, kind="native") for _ in range(2)]
        inv = rx[0].tables()["inv_scale"]
        t0 = time.perf_counter()
        for t in range(n):
            oracle_frame(t, "native", rx)
        cpu_s = time.perf_counter() - t0
        # parity: the checker build (-ffp-contract=off), every output of every frame
        rx = [orbref.RefExtractor(args.nfeatures, 1.2, 8, 20, 7) for _ in range(2)]
        parts = {k: True for k in ("keypoints", "descriptors", "u_right", "motion_model", "local_points")}
        for t in range(n):
            g, c = outs[t], oracle_frame(t, "checker", rx)
            parts["keypoints"] &= bool(g[0].tobytes() == c[0].tobytes() and g[2].tobytes() == c[2].tobytes())
            parts["descriptors"] &= bool(np.array_equal(g[1], c[1]) and np.array_equal(g[3], c[3]))
            parts["u_right"] &= bool(np.array_equal(g[4].view(np.uint32), c[4].view(np.uint32)))
            parts["motion_model"] &= bool((g[5], g[7]) == (c[5], c[7]) and np.array_equal(g[6], c[6]))
            parts["local_points"] &= bool((g[8], g[10]) == (c[8], c[10]) and np.array_equal(g[9], c[9]))
        out["cpu_baseline"] = {"value": round(n / cpu_s, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"the same sequence on the first {n} frames, oracle -O3 -march=native, 1 thread "
                                         "(the stereo Frame's two extractions serial here)"}
        out["cpu_bit_exact"] = all(parts.values())
        out["cpu_parity"] = parts
    return out


def c5_pmc_traffic(m_points):
    """HBM bytes of one SearchLocalPoints call's kernels (isInFrustum + SearchByProjection) from the
    committed rocprofv3 PMC summary (profiles/pmc_traffic_c5.json, profiles/scripts/c5_only.py), or
    None when none is committed for this map size."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic_c5.json")) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    if doc.get("workload", {}).get("map_points") != m_points:
        return None
    return int(doc["traffic_bytes_per_search"])


def pairing_leg(args, exts, tree, voc, d_img, pstreams, dev, subbatches=256):
    """The C3 step with the other SearchForTriangulation pairing on the same resident frames and
    handles (--pairs kf runs: left_i vs right_i of each frame with ComputeBoW on all 2B images, the
    rounds 1-2 workload; --pairs stereo runs: KeyFrame t vs t+1): `subbatches` sub-batches timed
    wall-clock after a warm-up, and its SearchForTriangulation matches per pair. Reported beside
    `value`, which is the default pairing's."""
    import torch
    from orb_slam2_2021_amd.pipeline import build_c3
    other = "stereo" if args.pairs == "kf" else "kf"
    B, H, W = args.batch, args.rows, args.cols
    pipe, _ = build_c3(exts if len(exts) > 1 else exts[0], tree, voc, B, H, W, dev, seed=1234,
                       depth=pipe_depth(args), stereo=args.stereo, levelsup=args.levelsup, streams=pstreams,
                       pairs=other, stereo_on_match=not args.stereo_on_extract)
    torch.cuda.set_stream(pipe.stream)
    nb = d_img.shape[0]
    for j in range(16):
        pipe.run(d_img[j % nb].data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(subbatches):
        pipe.run(d_img[j % nb].data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nm = pipe.last.nm.cpu().numpy()[:pipe.n_pairs]
    return {"pairs": other, "value": round(B * subbatches / dt, 1), "unit": "stereo frames/s",
            "sft_pairs_per_subbatch": pipe.n_pairs, "sft_matches_per_pair": round(float(nm.mean()), 1),
            "what": f"{subbatches} sub-batches of the C3 step with pairs={other} on the same frames and handles"}


def keyframe_leg(args, reps=20):
    """Secondary measurement: the remaining ORBmatcher searches and
    MapPoint::ComputeDistinctiveDescriptors on a KITTI-shaped keyframe scene (two KeyFrames of
    ~2000 keypoints over 1500 shared world points, synthetic vocabulary k=10, L=2), each through
    its host-buffer C ABI entry (inputs uploaded and results returned every call: PCIe included),
    beside the CPU oracle (-O3 -march=native, one core) on the same inputs and a bit-exact check.
    Wall-clock per call on both sides; reported, not `value`."""
    from orb_slam2_2021_amd import ORBmatcher
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import KeyFrameMapPoints
    from oracle import orbref
    rng = np.random.default_rng(0x0B0C)
    voc = S.Vocabulary.synthetic()
    sc = S.make_keyframe_scene(rng, n_points=1500, n_clutter=500, vocab=voc)
    kfs = [sc.kf2] + [S.make_keyframe_scene(np.random.default_rng(s), n_points=1500, n_clutter=500,
                                            vocab=voc).kf2 for s in range(1, 8)]
    cur = sc.f1
    cur_state = cur.mp_state.copy()
    sparse = np.where(rng.random(cur.N) < 0.2, 1, 0).astype(np.uint8)
    pts = KeyFrameMapPoints(sc.mps2, sc.kf2.keys_un["angle"])
    Scw = np.vstack([sc.kf1.tcw, [0, 0, 0, 1]]).astype(np.float32)
    Scw[:3] *= np.float32(0.9)
    s12, R12, t12 = S.sim3_between(sc.kf1.tcw, sc.kf2.tcw, 1.0)
    prev = np.stack([cur.keys_un["x"], cur.keys_un["y"]], 1).astype(np.float32)
    sets = S.distinctive_sets(rng, 2000, max_obs=20)
    m = ORBmatcher(0.75, True)
    mi = ORBmatcher(0.9, True)  # Initializer's matcher (Tracking::MonocularInitialization)

    def with_state(state, fn):
        def run():
            cur.mp_state = state
            try:
                return fn()
            finally:
                cur.mp_state = cur_state
        return run

    cases = {
        "SearchByBoW(KF,F)": (lambda: m.SearchByBoW(sc.kf2, cur),
                              lambda k: orbref.search_by_bow(sc.kf2, cur, 0.75, True, False, kind=k)),
        "SearchByBoW(KF,KF)": (lambda: m.SearchByBoW(sc.kf1, sc.kf2),
                               lambda k: orbref.search_by_bow(sc.kf1, sc.kf2, 0.75, True, True, kind=k)),
        "SearchByBoW x8 KFs (relocalisation)": (
            lambda: m.SearchByBoWMulti(kfs, cur),
            lambda k: [orbref.search_by_bow(kf, cur, 0.75, True, False, kind=k) for kf in kfs]),
        "SearchByProjection(F,KF)": (
            with_state(sparse, lambda: m.SearchByProjection(cur, sc.kf2, pts, 10, 100)),
            lambda k: with_state(sparse, lambda: orbref.search_by_projection_keyframe(cur, pts, 10, 100, True,
                                                                                     kind=k))()),
        "SearchByProjection(KF,Scw)": (lambda: m.SearchByProjection(sc.kf1, Scw, sc.mps2, 10),
                                       lambda k: orbref.search_by_projection_sim3(sc.kf1, Scw, sc.mps2, 10,
                                                                                  kind=k)),
        "Fuse(KF)": (lambda: m.Fuse(sc.kf1, sc.mps2, 3.0), lambda k: orbref.fuse(sc.kf1, sc.mps2, 3.0, kind=k)),
        "Fuse(KF,Scw)": (lambda: m.Fuse(sc.kf1, Scw, sc.mps2, 4.0),
                         lambda k: orbref.fuse_sim3(sc.kf1, Scw, sc.mps2, 4.0, kind=k)),
        "SearchBySim3": (lambda: m.SearchBySim3(sc.kf1, sc.kf2, sc.mps1, sc.mps2, s12, R12, t12, 7.5),
                         lambda k: orbref.search_by_sim3(sc.kf1, sc.kf2, sc.mps1, sc.mps2, s12, R12, t12, 7.5,
                                                         kind=k)),
        "SearchForInitialization": (lambda: mi.SearchForInitialization(cur, sc.f2, prev, 100),
                                    lambda k: orbref.search_for_initialization(cur, sc.f2, prev, 100, 0.9, True,
                                                                               kind=k)),
        "ComputeDistinctiveDescriptors x2000": (lambda: m.ComputeDistinctiveDescriptors(sets),
                                               lambda k: orbref.compute_distinctive_descriptors(sets, kind=k)),
    }

    out = {}
    for name, (gpu, cpu) in cases.items():
        g = gpu()
        t0 = time.perf_counter()
        for _ in range(reps):
            gpu()
        gms = 1e3 * (time.perf_counter() - t0) / reps
        row = {"gpu_ms_per_call": round(gms, 3)}
        if not args.no_cpu:
            t0 = time.perf_counter()
            c = cpu("native")
            row["cpu_oracle_ms_per_call"] = round(1e3 * (time.perf_counter() - t0), 3)
            if name.startswith("SearchByBoW x8"):
                gc, go = g
                same = all(int(gc[i]) == c[i][0] and np.array_equal(go[i], c[i][1]) for i in range(len(kfs)))
            elif name.startswith("SearchForInitialization"):
                same = g[0] == c[0] and np.array_equal(g[1], c[1]) and np.array_equal(g[2], c[2])
            elif name.startswith("ComputeDistinctive"):
                same = np.array_equal(g, c)
            else:
                same = g[0] == c[0] and np.array_equal(g[1], c[1])
            row["cpu_bit_exact"] = bool(same)
        out[name] = row
    out["what"] = ("host-buffer C ABI call per search (upload, kernels, download) on a KITTI-shaped keyframe "
                   "scene (~2000 keypoints per KeyFrame), 1 GPU; CPU oracle one core")
    return out


def stereo_leg(args, ext, d_img, host, B, H, W, cap, mbf, mb, reps=30):
    """Secondary measurement: Frame::ComputeStereoMatches on the step's B
    pairs, device-resident, after one extraction of the 2B images (the pyramids it reads stay in
    HBM). GPU: HIP events around `reps` launches of the 3-kernel sequence on the extraction stream;
    roofline of that sequence (algorithmic bytes per pair: both sides' keypoints + descriptors,
    2 x 16 B right-keypoint buckets, 12 B out per left keypoint). CPU: the oracle built with the
    reference's flags on one core, on the same pairs. Parity: the GPU output of every pair is
    compared with the oracle run on the GPU's keypoints and pyramid levels."""
    import torch
    from oracle import orbref
    from orb_slam2_2021_amd import _lib as L
    dev = d_img.device
    n_img = 2 * B
    kps = torch.empty(n_img * cap * 28, dtype=torch.uint8, device=dev)
    desc = torch.empty(n_img * cap * 32, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n_img, dtype=torch.int32, device=dev)
    ur = torch.empty(B * cap, dtype=torch.float32, device=dev)
    dep = torch.empty(B * cap, dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)
    s = stream.cuda_stream

    def run():
        ext.compute_stereo_matches_batch_device(B, 0, B, kps.data_ptr(), desc.data_ptr(),
                                                cnt.data_ptr(), cap, mbf, mb, ur.data_ptr(),
                                                dep.data_ptr(), stream=s)

    with torch.cuda.stream(stream):
        ext.extract_batch_device(n_img, d_img.data_ptr(), H * W, H, W, W, kps.data_ptr(),
                                 desc.data_ptr(), cap, cnt.data_ptr(), stream=s)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    K = kps.cpu().numpy().view(L.KEYPOINT_DTYPE)
    D = desc.cpu().numpy().reshape(-1, 32)
    C = cnt.cpu().numpy()
    UR, DEP = ur.cpu().numpy(), dep.cpu().numpy()
    matches, same, cpu_s = 0, True, 0.0
    scale, inv = ext.GetScaleFactors(), ext.GetInverseScaleFactors()
    for p in range(B):
        nl, nr = int(C[p]), int(C[B + p])
        kl, dl = K[p * cap:p * cap + nl], D[p * cap:p * cap + nl]
        kr, dr = K[(B + p) * cap:(B + p) * cap + nr], D[(B + p) * cap:(B + p) * cap + nr]
        pl = [ext.level(lv, image=p) for lv in range(ext.nlevels)]
        pr = [ext.level(lv, image=B + p) for lv in range(ext.nlevels)]
        t0 = time.perf_counter()
        wu, wd = orbref.compute_stereo_matches(kl, dl, kr, dr, pl, pr, scale, inv, mb, mbf,
                                               kind="native")
        cpu_s += time.perf_counter() - t0
        gu, gd = UR[p * cap:p * cap + nl], DEP[p * cap:p * cap + nl]
        same &= bool(np.array_equal(gu.view(np.uint32), wu.view(np.uint32))
                     and np.array_equal(gd.view(np.uint32), wd.view(np.uint32)))
        matches += int((gu >= 0).sum())
    nkp = int(C.sum())
    algo = 60 * nkp + 32 * nkp // 2 + 12 * nkp // 2  # bytes per launch sequence (B pairs)
    achieved = algo / (us * 1e-6) / 1e9
    return {
        "pairs_per_s": round(B / (us * 1e-6), 1), "us_per_batch": round(us, 2), "batch_pairs": B,
        "stereo_matches_per_pair": round(matches / B, 1),
        "parity_all_pairs_bit_exact": same,
        "roofline": {"kernel": "k_stereo_rows + k_stereo_match + k_stereo_median", "bound": "hbm",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": stereo_traffic(args, W, H, B),
                     "traffic_what": "PMC HBM bytes of the three stereo kernels per launch sequence (B pairs), "
                                     "profiles/pmc_traffic.json",
                     "algorithmic_bytes_per_launch_sequence": algo},
        "cpu_baseline": {"value": round(B / cpu_s, 1), "unit": "pairs/s", "cores": 1, "kind": "port",
                         "sample": f"ComputeStereoMatches oracle (-O3 -march=native) on the same {B} "
                                   f"pairs' keypoints and pyramids, 1 thread"},
        "what": "device-resident batch after extraction; events around the 3 stereo launches",
    }


def stereo_traffic(args, W, H, B):
    """PMC HBM bytes of one ComputeStereoMatches launch sequence (k_stereo_rows + k_stereo_match +
    k_stereo_median over B pairs), from the bench workload's committed summary, or None."""
    tot = 0
    for k in ("k_stereo_rows", "k_stereo_match", "k_stereo_median"):
        t, _ = pmc_traffic(k, W, H, B, args)
        if t is None:
            return None
        tot += t
    return tot


def vocab_leg(args, voc, tree, pipe, reps=20):
    """KeyFrame::ComputeBoW alone: the vocabulary transform of the last
    sub-batch's KeyFrame descriptor sets (the B lefts with --pairs kf; BowVector + FeatureVector,
    L=6 tree, levelsup 4), HIP events
    around `reps` device launches; the oracle (std::map containers, one core) on the same sets."""
    import torch
    o = pipe.last
    s = pipe.mstream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        voc.transform_batch_device(pipe.n_vocab, o.desc.data_ptr(), pipe.cap * 32, o.cnt.data_ptr(),
                                   pipe.levelsup, o.ids.data_ptr(), o.offs.data_ptr(), o.idx.data_ptr(),
                                   o.nodes.data_ptr(), pipe.cap, stream=s.cuda_stream,
                                   d_bow_words=o.bow_words.data_ptr(), d_bow_weights=o.bow_weights.data_ptr(),
                                   d_bow_n=o.bow_n.data_ptr())

    torch.cuda.synchronize()
    run()
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nkp = int(o.cnt[:pipe.n_vocab].sum().item())
    out = {"us_per_subbatch": round(us, 2), "descriptor_sets": pipe.n_vocab, "descriptors": nkp,
           "tree_nodes": tree.n_nodes, "descriptors_per_s": round(nkp / (us * 1e-6), 1)}
    if not args.no_cpu:
        from oracle.orbref import RefVocabulary
        ref = RefVocabulary.from_table(tree.k, tree.levels, tree.scoring, tree.weighting, tree.parent,
                                       tree.is_leaf, tree.descriptors, tree.weights)
        host = pipe.to_host(o)
        t0 = time.perf_counter()
        same = True
        for i in range(pipe.n_vocab):
            w, wt, fv = ref.transform(host["descriptors"][i], pipe.levelsup)
            gw, gt = host["bow"][i]
            gi, go, gx = host["fv"][i]
            same &= bool(np.array_equal(w, gw) and np.array_equal(wt.view(np.uint64), gt.view(np.uint64))
                         and np.array_equal(fv[0], gi) and np.array_equal(fv[1], go) and np.array_equal(fv[2], gx))
        cpu_s = time.perf_counter() - t0
        out["cpu_oracle_us_per_subbatch"] = round(cpu_s * 1e6, 1)
        out["cpu_bit_exact"] = same
    return out


def host_boundary_rate(ext, host, reps=20, others=()):
    """PCIe-inclusive extraction rate through the host-buffer C ABI entry orbfe_extract_batch on
    the step's 64 host images, with preallocated output buffers as a C++ caller keeps them.
    Reported beside `value`, never as it. Wall clock per call, two ways:
      staged      -- plain caller memory: pinned staging by the handle's worker threads, chunked
                     H2D / extraction / D2H on overlapping streams, used slots unpacked;
      registered  -- the caller's image and output buffers page-locked once (orbfe_host_register):
                     images DMA'd straight from them, results DMA'd straight into them.
    pcie_GBps = (image bytes in + keypoint/descriptor slot bytes out) / wall time."""
    from ctypes import c_size_t, c_void_p
    from orb_slam2_2021_amd import _lib as L
    from orb_slam2_2021_amd import register_host, unregister_host
    lib = L.lib()
    n, rows, cols = host.shape
    cap = ext.max_keypoints(rows, cols)
    kps = np.empty(n * cap, L.KEYPOINT_DTYPE)
    desc = np.empty((n * cap, 32), np.uint8)
    counts = np.zeros(n, np.int32)
    arr = (c_void_p * n)(*[host[i].ctypes.data for i in range(n)])

    def call():
        L.check(lib.orbfe_extract_batch(ext._h, n, ctypes.cast(arr, c_void_p), rows, cols, c_size_t(cols),
                                        L.ptr(kps), L.ptr(desc), cap, L.ptr(counts)), "orbfe_extract_batch")

    def timed():
        for _ in range(3):
            call()
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            call()
            times.append(time.perf_counter() - t0)
        return float(np.median(times))

    moved = host.nbytes + n * cap * (28 + 32)
    dt_staged = timed()
    staged = (kps[:counts[0]].copy(), desc[:counts[0]].copy(), counts.copy())
    hostc = np.ascontiguousarray(host)
    register_host(hostc)
    register_host(kps)
    register_host(desc)
    try:
        arr = (c_void_p * n)(*[hostc[i].ctypes.data for i in range(n)])
        dt_reg = timed()
        same = bool(np.array_equal(counts, staged[2]) and kps[:counts[0]].tobytes() == staged[0].tobytes()
                    and np.array_equal(desc[:counts[0]], staged[1]))
    finally:
        unregister_host(hostc)
        unregister_host(kps)
        unregister_host(desc)
    out = {"value": round(n / 2 / dt_reg, 2), "unit": "stereo frames/s", "ms_per_call_p50": round(1e3 * dt_reg, 3),
           "pcie_GBps": round(moved / dt_reg / 1e9, 2),
           "staged": {"value": round(n / 2 / dt_staged, 2), "ms_per_call_p50": round(1e3 * dt_staged, 3),
                      "pcie_GBps": round(moved / dt_staged / 1e9, 2)},
           "registered_equals_staged": same,
           "what": f"orbfe_extract_batch on {n} host images {cols}x{rows} (extract only; H2D + kernels + D2H; "
                   f"median of {reps} calls): value = caller buffers registered (orbfe_host_register, direct DMA), "
                   "staged = plain caller memory through the handle's pinned staging"}
    if others:
        out["threads"] = host_threads([ext] + list(others), hostc, cap, reps)
    return out


def host_threads(exts, host, cap, reps):
    """The host boundary with several extractor handles on as many threads, registered buffers:
      left_right  -- Frame.cc:113-116's own threading: per call pair, one thread extracts the B left
                     images and another the B right images (orbfe_extract_batch each), joined;
      streamed_N  -- N callers (2, and every handle), each extracting all 2B images per call back to
                     back into its own output buffers, so one caller's H2D overlaps another's kernels.
    Both in stereo frames/s over wall time (median per joined pair / total over the run)."""
    from concurrent.futures import ThreadPoolExecutor
    from ctypes import c_size_t, c_void_p
    from orb_slam2_2021_amd import _lib as L
    from orb_slam2_2021_amd import register_host, unregister_host
    lib = L.lib()
    n, rows, cols = host.shape
    B = n // 2

    class Caller:
        def __init__(self, h, imgs):
            self.h, self.m = h, len(imgs)
            self.kps = np.empty(self.m * cap, L.KEYPOINT_DTYPE)
            self.desc = np.empty((self.m * cap, 32), np.uint8)
            self.counts = np.zeros(self.m, np.int32)
            self.arr = (c_void_p * self.m)(*[im.ctypes.data for im in imgs])
            register_host(self.kps)
            register_host(self.desc)

        def __call__(self, k=1):
            for _ in range(k):
                L.check(lib.orbfe_extract_batch(self.h, self.m, ctypes.cast(self.arr, c_void_p), rows, cols,
                                                c_size_t(cols), L.ptr(self.kps), L.ptr(self.desc), cap,
                                                L.ptr(self.counts)), "orbfe_extract_batch")

        def close(self):
            unregister_host(self.kps)
            unregister_host(self.desc)

    register_host(host)
    pool = ThreadPoolExecutor(max_workers=len(exts))
    callers = []
    ext0 = exts[0]
    ext0.debug_set_blur_mode(1)  # the several-handle placement (the blur after DistributeOctTree)
    out = {}
    try:
        lr = [Caller(exts[0]._h, [host[i] for i in range(B)]), Caller(exts[1]._h, [host[B + i] for i in range(B)])]
        st = [Caller(e._h, list(host)) for e in exts]
        callers = lr + st

        def run_all(group, k=1):
            fs = [pool.submit(c, k) for c in group]
            for f in fs:
                f.result()

        for _ in range(3):
            run_all(lr)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            run_all(lr)
            times.append(time.perf_counter() - t0)
        dt_lr = float(np.median(times))
        out["left_right"] = {"value": round(B / dt_lr, 2), "ms_per_frame_batch_p50": round(1e3 * dt_lr, 3)}
        for m in sorted({2, len(exts)}):
            run_all(st[:m], 2)
            t0 = time.perf_counter()
            run_all(st[:m], reps)
            dt = time.perf_counter() - t0
            out[f"streamed_{m}"] = {"value": round(m * reps * B / dt, 2), "ms_per_call": round(1e3 * dt / reps, 3),
                                    "pcie_GBps": round(m * reps * (host.nbytes + n * cap * 60) / dt / 1e9, 2)}
        out["counts_equal"] = bool(all(np.array_equal(c.counts, st[0].counts) for c in st)
                                   and np.array_equal(np.concatenate([lr[0].counts, lr[1].counts]), st[0].counts))
    finally:
        pool.shutdown()
        for c in callers:
            c.close()
        unregister_host(host)
        ext0.debug_set_blur_mode(0)
    out["what"] = (f"handles on threads, registered buffers: left_right = {B} lefts and {B} rights extracted "
                   "concurrently by two handles (Frame.cc:113-116), median of the joined pairs; streamed_N = N "
                   f"callers each extracting all {n} images per call back to back ({reps} calls each), total over "
                   "wall time; one 30 MB H2D copy runs at ~53 GB/s on this link (profiles/scripts/h2d_bw.py)")
    return out


def _cpu_name():
    import platform
    cpu = platform.processor() or "x86_64"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def cpu_threads(args):
    """Threads for the all-core CPU baseline: --cpu-threads, else the CPUs this process may run on
    (os.sched_getaffinity), capped by OMP_NUM_THREADS when the environment sets it (a GPU box
    grants a job a share of a larger machine and says so there: 16 for one GPU)."""
    if args.cpu_threads > 0:
        return args.cpu_threads, "--cpu-threads"
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (affinity mask: {aff} CPUs)"
    return aff, f"affinity mask ({aff} CPUs)"


def cpu_baseline(host, B, H, W, args, tree, state):
    """The oracle built with the reference's flags (-O3 -march=native, CMakeLists.txt:10-11) on the
    host's cores, three ways. Per stereo frame, the same work as the GPU step: the
    stereo Frame (extract left + right, Frame::ComputeStereoMatches on their pyramids), ComputeBoW
    of the KeyFrame, and SearchForTriangulation against the previous KeyFrame of the sequence
    (--pairs kf; with --pairs stereo: ComputeBoW of both images, SearchForTriangulation(left, right)):
      1 thread        -- the latency of one frame on one core;
      2 threads       -- the stereo Frame pattern (Frame.cc:113-116): left and right extracted on
                         two threads, then the rest;
      all cores       -- cpu_threads() independent streams of frames.
    `value` is the all-core rate. The oracle is a scalar restatement, not OpenCV's SIMD FAST /
    resize / GaussianBlur, so it understates the real reference's speed. Plus C1: 100 distinct
    synthetic stereo frames through the 2-thread extraction (the CPU-only config)."""
    from oracle import orbref
    from orb_slam2_2021_amd import synth_frame
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import FeatureVector
    ref_voc = orbref.RefVocabulary.from_table(tree.k, tree.levels, tree.scoring, tree.weighting, tree.parent,
                                              tree.is_leaf, tree.descriptors, tree.weights)
    cam, F12, (ex, ey) = state["cam"], state["F12"], state["epipole"]
    ur, mp = state["u_right"], state["mp_state"]
    kf_pairs = args.pairs == "kf"

    def new_extractors():
        return [orbref.RefExtractor(args.nfeatures, 1.2, 8, 20, 7, kind="native") for _ in range(2)]

    def keyframe(i, k, d, with_bow):
        d = d if d is not None else np.zeros((0, 32), np.uint8)
        F = S.Frame(keys_un=k, descriptors=d, u_right=ur[i, :len(k)], mp_state=mp[i, :len(k)],
                    scale_factors=state["scale"], level_sigma2=state["sigma2"], min_x=0.0, max_x=float(W),
                    min_y=0.0, max_y=float(H), **cam)
        if with_bow:
            _, _, fv = ref_voc.transform(d, args.levelsup)
            F.feat_vec = FeatureVector(*fv)
        return F

    def frame_work(ext, p, k1, d1, k2, d2, prev):
        """Everything after the two extractions; returns this frame's left KeyFrame."""
        F1 = keyframe(p, k1, d1, True)
        F2 = keyframe(B + p, k2, d2, not kf_pairs)
        if args.stereo:
            lv = [ext[0].level(i) for i in range(8)]
            rv = [ext[1].level(i) for i in range(8)]
            F1.u_right, _ = orbref.compute_stereo_matches(F1.keys_un, F1.descriptors, F2.keys_un, F2.descriptors,
                                                          lv, rv, state["scale"], ext[0].tables()["inv_scale"], state["mb"],
                                                          cam["bf"], kind="native")
        if not kf_pairs:
            orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, False)
        elif prev is not None:
            orbref.search_for_triangulation(prev, F1, F12, ex, ey, False, False)
        return F1

    def stream(n_threads_inner, budget, first, stats, lock):
        ext = new_extractors()
        frames, t_total, prev = 0, 0.0, None
        while t_total < budget or frames < 2:
            p = (first + frames) % B
            if p == 0:
                prev = None  # the batch wraps: frame 0 does not follow frame B-1
            t0 = time.perf_counter()
            if n_threads_inner == 2:
                out = [None, None]
                t = threading.Thread(target=lambda: out.__setitem__(1, ext[1](host[B + p])))
                t.start()
                out[0] = ext[0](host[p])
                t.join()
                (k1, d1), (k2, d2) = out
            else:
                k1, d1 = ext[0](host[p])
                k2, d2 = ext[1](host[B + p])
            prev = frame_work(ext, p, k1, d1, k2, d2, prev)
            t_total += time.perf_counter() - t0
            frames += 1
        with lock:
            stats.append((frames, t_total))

    modes = {}
    lock = threading.Lock()
    for name, inner in (("1_thread", 1), ("2_threads_stereo", 2)):
        st = []
        stream(inner, args.cpu_seconds, 0, st, lock)
        f, t = st[0]
        modes[name] = {"stereo_frames_per_s": round(f / t, 3), "ms_per_frame": round(1e3 * t / f, 2),
                       "frames": f, "threads": inner}
    T, why = cpu_threads(args)
    st = []
    th = [threading.Thread(target=stream, args=(1, args.cpu_seconds, (i * 7) % B, st, lock)) for i in range(T)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    all_frames = sum(f for f, _ in st)
    modes["all_cores"] = {"stereo_frames_per_s": round(all_frames / wall, 3), "frames": all_frames,
                          "threads": T, "threads_from": why, "wall_s": round(wall, 2)}
    # C1: 100 distinct stereo frames, extraction only, the stereo Frame's two threads
    ext = new_extractors()
    t0 = time.perf_counter()
    for i in range(100):
        l, r = synth_frame(10_000 + i, H, W, right=True)
        t = threading.Thread(target=lambda: ext[1](r))
        t.start()
        ext[0](l)
        t.join()
    c1 = time.perf_counter() - t0
    work = ("2 x ORBextractor" + (" + ComputeStereoMatches" if args.stereo else "")
            + (f" + ComputeBoW (k=10 L={tree.levels}) + SearchForTriangulation(previous KF, KF)" if kf_pairs
               else f" + 2 x ComputeBoW (k=10 L={tree.levels}) + SearchForTriangulation(left, right)"))
    return {"value": modes["all_cores"]["stereo_frames_per_s"], "unit": "stereo frames/s", "cores": T,
            "kind": "port",
            "sample": f"{all_frames} stereo frames over {T} threads (each cycling this rank's {B} frames) "
                      f"{W}x{H}: {work} per frame, on {_cpu_name()}; oracle built -O3 -march=native -- a scalar "
                      "restatement, not OpenCV's SIMD FAST/resize/GaussianBlur, so it understates the reference",
            "modes": modes,
            "c1_100_frames": {"seconds": round(c1, 2), "ms_per_stereo_frame": round(10 * c1, 2),
                              "what": "100 distinct synthetic KITTI-shaped stereo frames, ORBextractor on "
                                      "left + right on two threads (Frame.cc:113-116), oracle -O3 -march=native"}}


if __name__ == "__main__":
    main()
