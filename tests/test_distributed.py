"""The N>1 path on CPU: world_size-2 gloo processes shard frames, extract with the CPU oracle
(standing in for the GPU extractor, which needs a device) and gather every rank's results to
rank 0 through the same gather_to_root the benchmark uses over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from orb_slam2_2021_amd.parallel import gather_to_root, pack, shard_frames, unpack

N_FRAMES, ROWS, COLS, CAP = 5, 200, 300, 700


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from orb_slam2_2021_amd import synth_frame
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    mine = shard_frames(N_FRAMES, world, rank)
    per_rank = -(-N_FRAMES // world)
    results = [ref(synth_frame(i, ROWS, COLS)) for i in mine]
    while len(results) < per_rank:  # pad to the common per-rank capacity
        results.append((np.zeros(0, results[0][0].dtype), None))
    c, k, d = pack(results, CAP)
    out = gather_to_root(torch.from_numpy(c), torch.from_numpy(k), torch.from_numpy(d))
    if rank == 0:
        frames = []
        for r in range(world):
            got = unpack(out[0][r].numpy(), out[1][r].numpy(), out[2][r].numpy(), CAP)
            frames.extend(got[:len(shard_frames(N_FRAMES, world, r))])
        q.put([(f[0].tobytes(), f[1].tobytes()) for f in frames])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_frames_partition():
    for n in (0, 1, 7, 512):
        for world in (1, 2, 3, 8):
            parts = [shard_frames(n, world, r) for r in range(world)]
            assert [i for p in parts for i in p] == list(range(n))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_pack_unpack_roundtrip():
    from orb_slam2_2021_amd import KEYPOINT_DTYPE
    rng = np.random.default_rng(0)
    res = []
    for n in (0, 3, 17):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.random(n)
        res.append((k, rng.integers(0, 256, (n, 32), dtype=np.uint8)))
    back = unpack(*pack(res, 20), 20)
    for (k0, d0), (k1, d1) in zip(res, back):
        assert np.array_equal(k0, k1) and np.array_equal(d0, d1)


def test_gloo_two_rank_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from orb_slam2_2021_amd import synth_frame
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    assert len(got) == N_FRAMES
    for i, (kb, db) in enumerate(got):
        k, d = ref(synth_frame(i, ROWS, COLS))
        assert kb == k.tobytes() and db == d.tobytes()
