#!/usr/bin/env python3
"""Benchmark: ORB extract + match on synthetic 1241x376 KITTI-shaped stereo frames.

One step = one batch of B stereo frames per GPU (BASELINE.json configs[2], "C3"), inputs already
resident in HBM:
  1. ORBextractor::operator() on all 2B images        (k_resize x7, k_fast, k_octree, k_describe)
  2. vocabulary descent -> FeatureVector for each image (k_vocab; KeyFrame::ComputeBoW's half)
  3. ORBmatcher::SearchForTriangulation(left_i, right_i) for the B pairs        (k_sft)
  4. with N > 1 GPUs: RCCL gather of every rank's keypoints + descriptors to rank 0 (config C4)
value = stereo frames processed by all ranks / max-over-ranks wall time of the K timed steps.

Launch: python bench.py [--gpus 1] [--steps K] [--warmup W]; N > 1 via torch.distributed.run.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec (ORB extract+match) on 1241×376, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=32, help="stereo frames per GPU per step")
    p.add_argument("--rows", type=int, default=376)
    p.add_argument("--cols", type=int, default=1241)
    p.add_argument("--nfeatures", type=int, default=2000)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-gather", action="store_true")
    p.add_argument("--no-kernel-events", action="store_true")
    p.add_argument("--no-legs", action="store_true", help="skip the secondary C5 measurement")
    p.add_argument("--pipeline", type=int, default=2,
                   help="output sets in flight: 2 overlaps a step's matching with the next step's "
                        "extraction (1: strictly one step at a time)")
    p.add_argument("--stereo", action="store_true",
                   help="run Frame::ComputeStereoMatches on every pair after extraction (the stereo "
                        "Frame constructor's full path); its mvuRight feeds SearchForTriangulation")
    p.add_argument("--banded-pyramid", action="store_true",
                   help="one banded k_pyramid launch instead of per-level k_resize (comparison)")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from orb_slam2_2021_amd import ORBextractor, ORBmatcher, synth_frame
    from orb_slam2_2021_amd import _lib as L
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import epipole
    from orb_slam2_2021_amd.vocabulary import ORBVocabulary

    B, H, W = args.batch, args.rows, args.cols
    n_img = 2 * B
    # ---- inputs: B stereo frames of this rank, resident in HBM (lefts first, then rights) ----
    from orb_slam2_2021_amd.parallel import gather_to_root, shard_frames
    host = np.zeros((n_img, H, W), np.uint8)
    for i, idx in enumerate(shard_frames(world * B, world, rank)):
        l, r = synth_frame(idx, H, W, right=True)
        host[i], host[B + i] = l, r
    d_img = torch.from_numpy(host).to(dev)
    ext = ORBextractor(args.nfeatures, 1.2, 8, 20, 7, device=dev.index)
    if args.banded_pyramid:
        ext.debug_force_level_launches(False)
    cap = ext.max_keypoints(H, W)
    # ---- matcher inputs: vocabulary, per-keyframe stereo/MapPoint state, geometry ----
    tree = S.Vocabulary.synthetic()
    voc = ORBVocabulary.from_tree(tree, device=dev.index)
    rng = np.random.default_rng(1234 + rank)
    ur = np.where(rng.random((n_img, cap)) < 0.5, rng.uniform(10, 1200, (n_img, cap)), -1.0)
    d_ur = torch.from_numpy(ur.astype(np.float32)).to(dev)
    mp = np.where(rng.random((n_img, cap)) < 0.3, L.ORBFE_MP_OBSERVED, L.ORBFE_MP_NONE)
    d_mp = torch.from_numpy(mp.astype(np.uint8)).to(dev)
    scale = ext.GetScaleFactors()
    sigma2 = ext.GetScaleSigmaSquares()
    d_scale = torch.from_numpy(scale).to(dev)
    d_sigma2 = torch.from_numpy(sigma2).to(dev)
    cam = S.KITTI_CAM
    t1, t2 = S.pose(), S.pose(tx=-0.537, tz=0.05)
    F12 = S.compute_f12(t1, t2, S.intrinsics(cam))
    dummy = S.make_frame(np.zeros(0, L.KEYPOINT_DTYPE), None, scale, sigma2, H, W, cam, rng, tcw=t1)
    dummy2 = S.make_frame(np.zeros(0, L.KEYPOINT_DTYPE), None, scale, sigma2, H, W, cam, rng, tcw=t2)
    ex, ey = epipole(dummy, dummy2)

    # ---- output sets: the step's extraction writes set (step % depth) while the matching of the
    # previous step still reads the other one (a two-deep pipeline across steps; every step does
    # all of its work, the streams only overlap one step's matching with the next's extraction)
    depth = max(1, args.pipeline)

    class OutSet:
        def __init__(self):
            self.kps = torch.empty(n_img * cap * 28, dtype=torch.uint8, device=dev)
            self.desc = torch.empty(n_img * cap * 32, dtype=torch.uint8, device=dev)
            self.cnt = torch.zeros(n_img, dtype=torch.int32, device=dev)
            self.ids = torch.empty(n_img * cap, dtype=torch.int32, device=dev)
            self.offs = torch.empty(n_img * (cap + 1), dtype=torch.int32, device=dev)
            self.idx = torch.empty(n_img * cap, dtype=torch.int32, device=dev)
            self.nodes = torch.zeros(n_img, dtype=torch.int32, device=dev)
            self.m12 = torch.empty(B * cap, dtype=torch.int32, device=dev)
            self.nm = torch.zeros(B, dtype=torch.int32, device=dev)
            self.ur = torch.full((B * cap,), -1.0, dtype=torch.float32, device=dev)
            self.dep = torch.full((B * cap,), -1.0, dtype=torch.float32, device=dev)
            self.matcher = ORBmatcher(0.6, False, device=dev.index)  # LocalMapping.cc:219
            self.pairs = (L.sft_pair * B)()
            for i in range(B):
                p = self.pairs[i]
                p.kf1, p.kf2 = self.view(i), self.view(B + i)
                p.fv1, p.fv2 = self.fvec(i), self.fvec(B + i)
                for k, x in enumerate(F12.reshape(9)):
                    p.f12[k] = float(x)
                p.ex, p.ey = ex, ey
                p.match12 = self.m12.data_ptr() + i * cap * 4
                p.nmatches = self.nm.data_ptr() + i * 4
                p.kf1_n_dev = self.cnt.data_ptr() + i * 4
                p.kf2_n_dev = self.cnt.data_ptr() + (B + i) * 4
                p.fv1_nodes_dev = self.nodes.data_ptr() + i * 4
                p.fv2_nodes_dev = self.nodes.data_ptr() + (B + i) * 4
            self.extracted = torch.cuda.Event()
            self.matched = torch.cuda.Event()

        def view(self, i):
            v = L.frame_view()
            v.n = 0  # read on the device from cnt[i]
            v.keys_un = self.kps.data_ptr() + i * cap * 28
            # left keyframes take mvuRight from ComputeStereoMatches when it runs (--stereo)
            v.u_right = (self.ur.data_ptr() + i * cap * 4 if args.stereo and i < B
                         else d_ur.data_ptr() + i * cap * 4)
            v.descriptors = self.desc.data_ptr() + i * cap * 32
            v.mp_state = d_mp.data_ptr() + i * cap
            v.nlevels = 8
            v.scale_factors = d_scale.data_ptr()
            v.level_sigma2 = d_sigma2.data_ptr()
            v.min_x, v.max_x, v.min_y, v.max_y = 0.0, float(W), 0.0, float(H)
            v.grid_inv_w = float(dummy.grid_inv_w)
            v.grid_inv_h = float(dummy.grid_inv_h)
            v.fx, v.fy, v.cx, v.cy, v.bf = cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["bf"]
            v.b = float(dummy.mb)
            return v

        def fvec(self, i):
            f = L.feature_vector()
            f.n_nodes = min(cap, tree.k ** tree.levels)  # upper bound; the count is read on the device
            f.node_ids = self.ids.data_ptr() + i * cap * 4
            f.offsets = self.offs.data_ptr() + i * (cap + 1) * 4
            f.indices = self.idx.data_ptr() + i * cap * 4
            return f

    sets = [OutSet() for _ in range(depth)]
    lib = L.lib()
    gather = world > 1 and not args.no_gather

    ev = {k: [] for k in ("k_vocab", "k_sft", "k_stereo")}
    ev_sel = set()  # which of the two non-extractor kernels get events in this pass
    stream = torch.cuda.Stream(dev)   # extraction
    mstream = torch.cuda.Stream(dev)  # vocabulary + matching (+ gather)
    counter = [0]

    def step():
        o = sets[counter[0] % depth]
        counter[0] += 1
        stream.wait_event(o.matched)  # the matching that last read this set is done
        ext.extract_batch_device(n_img, d_img.data_ptr(), H * W, H, W, W, o.kps.data_ptr(),
                                 o.desc.data_ptr(), cap, o.cnt.data_ptr(), stream=stream.cuda_stream)
        if args.stereo:  # Frame.cc:125, on the extraction stream while the pyramids are current
            if "k_stereo" in ev_sel:
                s0 = torch.cuda.Event(enable_timing=True)
                s0.record(stream)
            ext.compute_stereo_matches_batch_device(B, 0, B, o.kps.data_ptr(), o.desc.data_ptr(),
                                                    o.cnt.data_ptr(), cap, cam["bf"], float(dummy.mb),
                                                    o.ur.data_ptr(), o.dep.data_ptr(),
                                                    stream=stream.cuda_stream)
            if "k_stereo" in ev_sel:
                s1 = torch.cuda.Event(enable_timing=True)
                s1.record(stream)
                ev["k_stereo"].append((s0, s1))
        o.extracted.record(stream)
        mstream.wait_event(o.extracted)
        ms = mstream.cuda_stream
        if "k_vocab" in ev_sel:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(mstream)
        voc.transform_batch_device(n_img, o.desc.data_ptr(), cap * 32, o.cnt.data_ptr(), 0,
                                   o.ids.data_ptr(), o.offs.data_ptr(), o.idx.data_ptr(),
                                   o.nodes.data_ptr(), cap, stream=ms)
        if "k_vocab" in ev_sel:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(mstream)
            ev["k_vocab"].append((e0, e1))
        if "k_sft" in ev_sel:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record(mstream)
        L.check(lib.orbfe_search_for_triangulation_batch_device(
            o.matcher._h, B, ctypes.cast(o.pairs, ctypes.c_void_p), 0, ctypes.c_void_p(ms)), "sft batch")
        if "k_sft" in ev_sel:
            e3 = torch.cuda.Event(enable_timing=True)
            e3.record(mstream)
            ev["k_sft"].append((e2, e3))
        if gather:  # C4: every rank's keypoints + descriptors to rank 0 over RCCL
            with torch.cuda.stream(mstream):
                gather_to_root(o.cnt, o.kps, o.desc, dst=0)
        o.matched.record(mstream)

    def kernel_times():
        kt = ext.kernel_times()
        for k in ("k_vocab", "k_sft", "k_stereo"):
            if ev[k]:
                kt[k] = (sum(a.elapsed_time(b) for a, b in ev[k]), len(ev[k]))
        return {k: v for k, v in kt.items() if v[1] > 0}

    def barrier():
        if world > 1:
            dist.barrier()

    # all work goes to two non-default streams (extraction / matching) ordered by events, so every
    # library call, torch event and RCCL collective of a step is ordered (a NULL stream would
    # select each handle's own stream)
    torch.cuda.set_stream(stream)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # probe pass (untimed): HIP events around every kernel -> per-kernel durations and the
    # dominant kernel
    probe_steps = max(3, min(args.steps, 10))
    ext.reset_kernel_times()
    ext.set_profiling(True)
    ev_sel.update(("k_vocab", "k_sft", "k_stereo"))
    for _ in range(probe_steps):
        step()
    torch.cuda.synchronize()
    probe = kernel_times()
    ext.set_profiling(False)
    ev_sel.clear()
    ev["k_vocab"].clear()
    ev["k_sft"].clear()
    ev["k_stereo"].clear()
    dominant = max(probe, key=lambda k: probe[k][0])
    # timed region: events only around the dominant kernel's launches
    ext.reset_kernel_times()
    if not args.no_kernel_events:
        if dominant in ext.KERNELS:
            ext.set_profiling([dominant])
        else:
            ev_sel.add(dominant)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    ext.set_profiling(False)
    ev_sel.clear()
    timed = kernel_times()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames = world * B * args.steps
    value = frames / elapsed
    counts = sets[0].cnt.cpu().numpy()
    cand = ext.debug_candidate_total()
    nm = sets[0].nm.cpu().numpy()
    geo = ext.geometry(H, W)
    roof = roofline(timed if dominant in timed else probe, dominant, geo, counts, cand, n_img,
                    args.steps if dominant in timed else probe_steps)
    roof["measured_in"] = "timed region" if dominant in timed else "probe pass (--no-kernel-events)"
    roof["traffic"], roof["traffic_source"] = pmc_traffic(dominant, W, H, B)
    algo_frame = pipeline_bytes_per_stereo_frame(geo, counts, B)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "stereo frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded KITTI-shaped stereo frames, orbfe_synth_frame; synthetic vocabulary)",
        "config": {
            "workload": f"C3: stereo extract + "
                        + ("ComputeStereoMatches + " if args.stereo else "")
                        + f"SearchForTriangulation, {W}x{H}, batch {B} stereo frames/GPU"
                        + (" + RCCL gather to rank 0 (C4)" if gather else ""),
            "nfeatures": args.nfeatures, "scale_factor": 1.2, "nlevels": 8, "ini_th_fast": 20,
            "min_th_fast": 7, "stereo_frames_per_gpu_per_step": B, "images_per_step_per_gpu": n_img,
            "parallelism": f"frame-sharded x{world}",
            "pipeline": f"{depth} output sets: step i's matching overlaps step i+1's extraction"
                        if depth > 1 else "one step at a time",
        },
        "roofline": roof,
        "pipeline_hbm": {
            "algorithmic_bytes_per_stereo_frame": int(algo_frame),
            "achieved_GBps": round(algo_frame * value / 1e9, 3),
            "frac_of_peak": round(algo_frame * value / 1e9 / HBM_PEAK_GBS, 6),
        },
        "kernels_ms_per_step": {k: round(v[0] / probe_steps, 4) for k, v in probe.items()},
        "keypoints_per_image": round(float(counts.mean()), 1),
        "sft_matches_per_pair": round(float(nm.mean()), 1),
        "stereo_matches_per_pair": (round(float((sets[0].ur >= 0).sum().item()) / B, 1)
                                    if args.stereo else None),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1:
        out["host_boundary"] = host_boundary_rate(ext, host)
        if not args.no_legs:
            out["legs"] = {"c5_search_local_points": sbp_leg(args),
                           "keyframe_searches": keyframe_leg(args),
                           "compute_stereo_matches": stereo_leg(args, ext, d_img, host, B, H, W, cap,
                                                                cam["bf"], float(dummy.mb))}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(host, B, H, W, args, tree, cam, F12, ex, ey,
                                           float(dummy.mb))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def level_pixels(geo):
    return [int(w) * int(h) for w, h in geo[:, :2]]


def roofline(kt, dom, geo, counts, n_cand, n_img, steps):
    """Roofline of the dominant kernel: ALGORITHMIC bytes per step / its HIP-event time per step
    (a kernel may run as several launches per step, e.g. k_resize once per level and k_fast as
    level 0 beside the resize chain + levels 1..7; per launch = per step / launches_per_step).
    Per-kernel algorithmic bytes (per step; DESIGN.md 'Roofline'):
      k_resize   sum_l>=1 (px_{l-1} + px_l) per image (read the source level once, write the level)
      k_fast     sum_l px_l per image + 4 B per FAST candidate + 4 B per cell count
      k_octree   2 x 4 B per candidate (gather + partition) + 4 B per survivor
      k_blur     2 x sum_l px_l per image (read each level once, write its blurred copy)
      k_copy0    2 x px_0 per image
      k_pyramid  2 x px_0 + sum_l>=1 px_l per image (read the input, write every level once)
      k_describe 4 B in + 60 B out per keypoint (+ 749 + 512 gathered bytes per keypoint, not
                 counted: they overlap between keypoints and come from L2)
      k_vocab    32 B in + 12 B out per descriptor
      k_sft      per pair 2 N (32 + 28 + 4) B (descriptors, keypoints, flags/uRight) + 4 N1 out
      k_stereo   per pair 2 N (28 + 32) B + 2 x 16 B per right keypoint (buckets) + 12 B per left
                 keypoint (the 11x11 windows and candidate descriptors come from L2)"""
    px = level_pixels(geo)
    ncells = int(geo[:, 2].sum())
    nkp = int(counts.sum())
    per_step = {
        "k_resize": n_img * sum(px[l - 1] + px[l] for l in range(1, len(px))),
        "k_fast": n_img * (sum(px) + 4 * ncells) + 4 * n_cand,
        "k_octree": 8 * n_cand + 4 * nkp,
        "k_describe": 64 * nkp + n_img * 0,  # + the patch pixels it gathers
        "k_blur": n_img * 2 * sum(px),
        "k_copy0": n_img * 2 * px[0],
        "k_pyramid": n_img * (2 * px[0] + sum(px[1:])),
        "k_vocab": 44 * nkp,
        "k_sft": 64 * nkp + 4 * nkp // 2,
        # ComputeStereoMatches (3 launches): both sides' keypoints + descriptors, right-keypoint
        # buckets written and read (16 B), u_right / depth / SAD out (12 B per left keypoint)
        "k_stereo": 60 * nkp + 32 * nkp // 2 + 12 * nkp // 2,
    }
    total_ms, launches = kt[dom]
    per_launch_steps = max(launches // max(steps, 1), 1)  # launches per step
    step_s = total_ms / 1e3 / max(steps, 1)
    achieved = per_step[dom] / step_s / 1e9
    return {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
            "algorithmic_bytes_per_step": int(per_step[dom]),
            "algorithmic_bytes_per_launch": int(per_step[dom] / per_launch_steps),
            "kernel_us_per_step": round(step_s * 1e6, 2),
            "avg_launch_us": round(step_s * 1e6 / per_launch_steps, 2),
            "launches_per_step": per_launch_steps}


def pmc_traffic(kernel, W, H, B):
    """HBM bytes per step of `kernel` from the committed rocprofv3 PMC summary of this workload
    (profiles/pmc_traffic.json, written by profiles/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of `bench.py --no-cpu`; FETCH_SIZE doubled per MI355X_MICROARCH.md), or None
    when no summary for this kernel and workload is committed."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None, None
    if doc.get("workload") != {"cols": W, "rows": H, "batch": B}:
        return None, None
    k = doc.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return int(k["traffic_bytes_per_step"]), doc.get("source")


def pipeline_bytes_per_stereo_frame(geo, counts, B):
    """per image sum_l px (read once) + sum_l>=1 px (write) + 60 B per keypoint;
    SearchForTriangulation per pair 2 N (32 + 28 + 4) + N/4 + 8 N."""
    px = level_pixels(geo)
    n_per_img = float(counts.mean())
    extract = sum(px) + sum(px[1:]) + 60 * n_per_img
    sft = 2 * n_per_img * 64 + 2 * n_per_img / 8 + 4 * 2 * n_per_img
    return 2 * extract + sft


def sbp_leg(args, m_points=50000, reps=20):
    """Secondary measurement (BASELINE config C5 shape): Tracking::SearchLocalPoints' hot part on a
    640x480 frame against 50k local MapPoints -- Frame::isInFrustum(pMP, 0.5) for every MapPoint,
    then ORBmatcher(0.8).SearchByProjection(F, vpLocalMapPoints, th=3) (Tracking.cc:1186-1213) --
    through the host-buffer C ABI orbfe_search_local_points (frame and MapPoint SoA uploaded every
    call, so PCIe is included), beside the CPU oracle on the same input (one core, -O3
    -march=native) and a bit-exact check of the two. Reported, not `value`."""
    from orb_slam2_2021_amd import ORBextractor, ORBmatcher, synth_frame
    from orb_slam2_2021_amd import synthetic as S
    from orb_slam2_2021_amd.frames import log_scale_factor
    ext = ORBextractor(args.nfeatures, 1.2, 8, 12, 7)  # arducam.yaml:126-127
    k, d = ext(synth_frame(7, 480, 640))
    rng = np.random.default_rng(0x50C0DE)
    F = S.make_frame(k, d, ext.GetScaleFactors(), ext.GetScaleSigmaSquares(), 480, 640,
                     S.ARDUCAM_CAM, rng, mp_frac=0.0, tcw=S.pose(tx=0.1, yaw=0.02))
    G = S.make_local_map(F, m_points, rng)
    m = ORBmatcher(0.8, True)  # Tracking.cc:1206
    nm, best, nv, _ = m.SearchLocalPoints(F, G, 3.0)
    t0 = time.perf_counter()
    for _ in range(reps):
        m.SearchLocalPoints(F, G, 3.0)
    gpu_s = (time.perf_counter() - t0) / reps
    out = {"frames_per_s": round(1.0 / gpu_s, 1), "ms_per_frame": round(1e3 * gpu_s, 3),
           "map_points": m_points, "in_view": int(nv), "keypoints": int(len(k)),
           "matches": int(nm),
           "what": "orbfe_search_local_points per call (H2D of frame + MapPoints, isInFrustum + "
                   "SearchByProjection kernels, D2H), 1 GPU"}
    if not args.no_cpu:
        from oracle import orbref
        lsf = log_scale_factor(1.2)
        orbref.lib("native")
        t0 = time.perf_counter()
        nr, br, nvr, _ = orbref.search_local_points(F, G, lsf, 3.0, 0.8, kind="native")
        out["cpu_oracle_ms_per_frame"] = round(1e3 * (time.perf_counter() - t0), 3)
        out["cpu_bit_exact"] = bool(nr == nm and nvr == nv and np.array_equal(br, best))
    return out


def keyframe_leg(args, reps=20):
    """Secondary measurement: the remaining ORBmatcher searches and
    MapPoint::ComputeDistinctiveDescriptors on a KITTI-shaped keyframe scene (two KeyFrames of
    ~2000 keypoints over 1500 shared world points, synthetic vocabulary k=10, L=2), each through
    its host-buffer C ABI entry (inputs uploaded and results returned every call: PCIe included),
    beside the CPU oracle (-O3 -march=native, one core) on the same inputs and a bit-exact check.
    Wall-clock per call on both sides; reported, not `value`."""
    from orb_slam2_2021_amd import ORBmatcher, MPF_SKIP
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

    def canon(r):  # (count, array) tuples / lists of them -> comparable arrays
        if isinstance(r, list):
            return [canon(x) for x in r]
        if isinstance(r, tuple):
            return tuple(np.asarray(x).tolist() if isinstance(x, np.ndarray) else x for x in r)
        return np.asarray(r).tolist()

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
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                     "algorithmic_bytes_per_launch_sequence": algo},
        "cpu_baseline": {"value": round(B / cpu_s, 1), "unit": "pairs/s", "cores": 1, "kind": "port",
                         "sample": f"ComputeStereoMatches oracle (-O3 -march=native) on the same {B} "
                                   f"pairs' keypoints and pyramids, 1 thread"},
        "what": "device-resident batch after extraction; events around the 3 stereo launches",
    }


def host_boundary_rate(ext, host, reps=5):
    """PCIe-inclusive extraction rate through the host-buffer entry (orbfe_extract_batch: H2D of
    the images, the same kernels, D2H of keypoints + descriptors). Reported beside `value`, never as
    it."""
    import torch
    imgs = [host[i] for i in range(len(host))]
    ext.extract_batch(imgs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ext.extract_batch(imgs)
    dt = time.perf_counter() - t0
    return {"value": round(reps * len(imgs) / 2 / dt, 2), "unit": "stereo frames/s",
            "what": f"orbfe_extract_batch on {len(imgs)} host images (extract only, H2D + D2H included)"}


def cpu_baseline(host, B, H, W, args, tree, cam, F12, ex, ey, mb):
    """The oracle built with the reference's flags (-O3 -march=native, CMakeLists.txt:10-11) timed
    on one host core: extract left + right (+ ComputeStereoMatches with --stereo), then
    SearchForTriangulation(left, right), per stereo frame, for about --cpu-seconds (the vocabulary
    descent is left out of the CPU timing)."""
    from oracle import orbref
    from orb_slam2_2021_amd import synthetic as S
    ref = orbref.RefExtractor(args.nfeatures, 1.2, 8, 20, 7, kind="native")
    ref_r = orbref.RefExtractor(args.nfeatures, 1.2, 8, 20, 7, kind="native")
    tab = ref.tables()
    rng = np.random.default_rng(5)
    t_total, frames = 0.0, 0
    while t_total < args.cpu_seconds or frames < 2:  # cycles over this rank's B frames
        l, r = host[frames % B], host[B + frames % B]
        t0 = time.perf_counter()
        k1, d1 = ref(l)
        k2, d2 = ref_r(r)
        t1 = time.perf_counter()
        if args.stereo:  # ComputeStereoMatches on the two extractors' pyramids (copies untimed)
            lv = [ref.level(i) for i in range(8)]
            rv = [ref_r.level(i) for i in range(8)]
            ts = time.perf_counter()
            orbref.compute_stereo_matches(k1, d1, k2, d2, lv, rv, tab["scale"], tab["inv_scale"],
                                          mb, cam["bf"], kind="native")
            t1 += time.perf_counter() - ts
        F1 = S.make_frame(k1, d1, tab["scale"], tab["sigma2"], H, W, cam, rng)
        F2 = S.make_frame(k2, d2, tab["scale"], tab["sigma2"], H, W, cam, rng)
        F1.feat_vec = tree.feature_vector(d1, 0)
        F2.feat_vec = tree.feature_vector(d2, 0)
        t2 = time.perf_counter()
        orbref.search_for_triangulation(F1, F2, F12, ex, ey, False, False)
        t3 = time.perf_counter()
        t_total += (t1 - t0) + (t3 - t2)
        frames += 1
    import platform
    cpu = platform.processor() or "x86_64"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(frames / t_total, 3), "unit": "stereo frames/s", "cores": 1,
            "kind": "port",
            "sample": f"{frames} stereo frames (cycling the step's {B}) {W}x{H} (2 x ORBextractor + "
                      + ("ComputeStereoMatches + " if args.stereo else "") + "SearchForTriangulation) on "
                      f"1 thread of {cpu}; oracle built -O3 -march=native",
            "seconds": round(t_total, 2)}


if __name__ == "__main__":
    main()
