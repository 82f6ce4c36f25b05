"""bench.py's reporting helpers on CPU: the roofline object carries the contract's keys with
consistent arithmetic, the committed PMC summary is found for the benchmark workload, and the
CLI defaults are N=1 with a short run."""
import os
import sys

from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# level geometry of 1241x376 / 8 levels / 1.2 (w, h, ncells per level; other columns unused here)
GEO = np.array([[1241, 376, 429], [1034, 313, 297], [862, 261, 196], [718, 218, 138],
                [598, 181, 95], [499, 151, 64], [416, 126, 42], [346, 105, 30]])
GEO = np.hstack([GEO, np.zeros((8, 4), np.int64)])


def test_roofline_object():
    counts = np.full(64, 2007, np.int32)
    kt = {"k_fast": (50 * 0.25, 100)}  # 50 steps, 2 launches per step, 0.25 ms per step
    pipe = SimpleNamespace(n_vocab=32, pair_idx=[(i, i + 1) for i in range(31)], n_pairs=31)
    r = bench.roofline(kt, "k_fast", GEO, counts, 13_000 * 64, 64, 50, pipe)  # 50 sub-batches
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["launches_per_subbatch"] == 2
    per_step = r["algorithmic_bytes_per_subbatch"]
    assert abs(r["achieved"] - per_step / 0.25e-3 / 1e9) < 0.05
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-5
    px = sum(int(w) * int(h) for w, h in GEO[:, :2])
    assert per_step == 64 * (px + 4 * int(GEO[:, 2].sum())) + 4 * 13_000 * 64
    # SearchForTriangulation bytes follow the pairing: 31 KeyFrame pairs (t, t+1) of 2007 keypoints
    kt = {"k_sft_nodes": (50 * 0.1, 50)}
    r = bench.roofline(kt, "k_sft_nodes", GEO, counts, 0, 64, 50, pipe)
    assert r["algorithmic_bytes_per_subbatch"] == 31 * (64 * 2 * 2007 + 4 * 2007)
    # every kernel of the C3 step has algorithmic bytes (the dominant one is chosen by device time)
    for k in ("k_copy0", "k_resize_win", "k_fast", "k_octree", "k_blur", "k_describe", "k_stereo_rows",
              "k_stereo_match", "k_stereo_median", "k_vocab_descend", "k_vocab", "k_sft_nodes", "k_sft_finish"):
        r = bench.roofline({k: (50 * 0.1, 50)}, k, GEO, counts, 13_000 * 64, 64, 50, pipe)
        assert r["algorithmic_bytes_per_subbatch"] > 0 and 0 < r["frac"] < 1, k


def test_committed_pmc_traffic_matches_workload():
    a = SimpleNamespace(pairs="kf", stereo=True)  # the bench default
    t, src = bench.pmc_traffic("k_fast", 1241, 376, 32, a)
    assert t is not None and t > 0 and "FETCH_SIZE" in src
    assert bench.pmc_traffic("k_fast", 640, 480, 32, a) == (None, None)  # other workload: not reported
    assert bench.pmc_traffic("k_fast", 1241, 376, 32, SimpleNamespace(pairs="stereo", stereo=False)) == (None, None)
    # the stereo leg's traffic: all three ComputeStereoMatches kernels are in the summary
    assert bench.stereo_traffic(a, 1241, 376, 32) > 0
    # C5: the search's kernels for the 50k-MapPoint map
    assert bench.c5_pmc_traffic(50000) > 0 and bench.c5_pmc_traffic(1000) is None


def test_cli_defaults():
    saved = sys.argv
    sys.argv = ["bench.py"]
    try:
        a = bench.parse()
    finally:
        sys.argv = saved
    assert a.gpus == 1 and 0 < a.steps <= 100 and 0 <= a.warmup <= 20 and a.batch == 32
    assert a.input_batches >= 4 and a.vocab_levels == 6 and a.levelsup == 4
    # two extractor handles, two output sets each
    assert a.extractors == 2 and a.handles_per_stream == 2 and bench.pipe_depth(a) == 8 and not a.stereo_on_extract
    # SURVEY 8(d)'s KeyFrame pairs with the stereo Frame's ComputeStereoMatches
    assert a.pairs == "kf" and a.stereo
    # a step is long enough to be seen (>= 1024 sub-batches of 32 stereo frames)
    assert a.batches_per_step * a.batch >= 32 * 1024


def test_hw_queue_setting():
    # several ranks: RCCL's stream gets a hardware queue of its own beside the four pipeline streams
    assert bench.hw_queue_setting(-1, 1) == 0
    assert bench.hw_queue_setting(-1, 2) == bench.HW_QUEUES_MULTI_RANK >= 5
    assert bench.hw_queue_setting(-1, 8) == bench.HW_QUEUES_MULTI_RANK
    assert bench.hw_queue_setting(0, 8) == 0  # the environment's
    assert bench.hw_queue_setting(4, 1) == 4
    assert bench.parse([]).hw_queues == -1 and bench.parse([]).c5_workers >= 1


def test_root_share_schedule():
    """C4's rank-0 share: the model and the slot schedule."""
    import bench
    assert bench.root_share(-1, 1) == 1.0
    assert abs(bench.root_share(-1, 8) - (1 - 7 * bench.ROOT_INGEST_PER_PEER)) < 1e-12
    assert bench.root_share(0.3, 8) == 0.3 and bench.root_share(2.0, 8) == 1.0
    for n, f in [(1024, 0.809), (1024, 1.0), (7, 0.5), (3, 0.97), (100, 0.0)]:
        own = bench.own_slots(n, f)
        assert len(own) == n and sum(own) == int(n * f + 0.5)
        if f > 0:
            assert own[0]  # the first slot runs rank 0's own sub-batch
    # the whole-job loss the share leaves at N = 8 (rank 0 and the peers finish together)
    f = bench.root_share(-1, 8)
    assert (1 - f) / 8 <= 0.05
