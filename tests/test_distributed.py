"""The N>1 path on CPU (world_size-2 gloo processes), through the same functions bench.py uses over
RCCL on GPUs:
* C4: ranks shard the frames, pack their used keypoints + descriptors (pack_host: the device
  packer's layout), and gather_packed moves sizes first, then only the used bytes, to rank 0;
* C5: rank 0's local map (MapPoint SoA) is replicated with broadcast_arrays and every rank runs
  its shard of frames against it; rank 0 collects every frame's matches;
* the launcher: bench.py --gpus N without a torch.distributed environment starts torchrun as a
  child (never an exec) and the ranks refuse a --gpus / WORLD_SIZE mismatch.
The extraction / search compute is the CPU oracle here (no device); GPU parity is tested in
tests/test_gpu_*.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from orb_slam2_2021_amd.parallel import (pack_host, packed_bytes, shard_frames, unpack_packed)

N_FRAMES, ROWS, COLS = 5, 200, 300
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _c4_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    from orb_slam2_2021_amd import synth_frame
    from orb_slam2_2021_amd.parallel import gather_packed
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    results = [ref(synth_frame(i, ROWS, COLS)) for i in shard_frames(N_FRAMES, world, rank)]
    buf = pack_host(results)
    payload = torch.zeros(packed_bytes(len(results), 600 * len(results)) + 64, dtype=torch.uint8)
    payload[:len(buf)] = torch.from_numpy(buf)
    size = torch.tensor([len(buf)], dtype=torch.int64)
    out, sizes = gather_packed(payload, size, dst=0)
    if rank == 0:
        frames = []
        for r in range(world):
            assert out[r].numel() == sizes[r]
            frames.extend(unpack_packed(out[r].numpy()))
        q.put(("c4", [(f[0].tobytes(), f[1].tobytes()) for f in frames], sizes))
    dist.barrier()
    dist.destroy_process_group()


def _c4_fixed_worker(rank, world, port, q):
    """bench.py's exchange: fixed byte count (the packed worst case), no size collective."""
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    from orb_slam2_2021_amd import synth_frame
    from orb_slam2_2021_amd.parallel import gather_fixed, packed_size
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    mine = shard_frames(N_FRAMES, world, rank)
    results = [ref(synth_frame(i, ROWS, COLS)) for i in mine]
    buf = pack_host(results)
    nbytes = packed_bytes(3, 3 * 600)  # every rank: the same worst case for 3 images of <= 600 kps
    payload = torch.full((nbytes,), 0xEE, dtype=torch.uint8)
    payload[:len(buf)] = torch.from_numpy(buf)
    out = gather_fixed(payload, nbytes, dst=0)
    if rank == 0:
        frames = []
        for r in range(world):
            assert out[r].numel() == nbytes
            v = out[r].numpy()
            frames.extend(unpack_packed(v[:packed_size(v)]))
        q.put(("c4f", [(f[0].tobytes(), f[1].tobytes()) for f in frames], None))
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def _c5_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    from orb_slam2_2021_amd.frames import MapPointGeometry
    from orb_slam2_2021_amd.parallel import broadcast_arrays, gather_packed
    from oracle import orbref
    scene = _c5_scene()
    G0, frames = scene
    fields = ("flags", "world_pos", "normal", "min_distance", "max_distance", "descriptors")
    arrs = {f: np.ascontiguousarray(getattr(G0, f)) for f in fields}
    if rank != 0:  # only rank 0 holds the map; the others receive it
        arrs = {f: np.zeros_like(a) for f, a in arrs.items()}
    got = broadcast_arrays(arrs, "cpu", src=0)
    G = MapPointGeometry(**{f: got[f].numpy().view(arrs[f].dtype).reshape(arrs[f].shape) for f in fields})
    res = []
    for i in shard_frames(len(frames), world, rank):
        nm, best, nv, _ = orbref.search_local_points(frames[i], G, 0.1823215568, 3.0, 0.8)
        res.append(np.concatenate([[i, nm, nv], best]).astype(np.int32))
    buf = np.concatenate(res).view(np.uint8)
    out, sizes = gather_packed(torch.from_numpy(buf.copy()), torch.tensor([len(buf)], dtype=torch.int64))
    if rank == 0:
        rows = np.concatenate([o.numpy().view(np.int32) for o in out])
        q.put(("c5", rows.tobytes(), len(frames)))
    dist.barrier()
    dist.destroy_process_group()


def _c5_scene():
    from orb_slam2_2021_amd import synth_frame
    from orb_slam2_2021_amd import synthetic as S
    from oracle.orbref import RefExtractor
    ext = RefExtractor(1000, 1.2, 8, 12, 7)
    tab = ext.tables()
    rng = np.random.default_rng(5)
    frames = []
    for i in range(3):
        k, d = ext(synth_frame(40 + i, 240, 320))
        frames.append(S.make_frame(k, d, tab["scale"], tab["sigma2"], 240, 320, S.ARDUCAM_CAM, rng, mp_frac=0.0,
                                   tcw=S.pose(tx=0.1 + 0.01 * i, yaw=0.02)))
    G = S.make_local_map(frames[0], 3000, np.random.default_rng(9))
    return G, frames


def _run(worker, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


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
    for n in (0, 3, 17, 0, 1):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.random(n)
        k["octave"] = rng.integers(0, 8, n)
        res.append((k, rng.integers(0, 256, (n, 32), dtype=np.uint8)))
    buf = pack_host(res)
    assert len(buf) == packed_bytes(5, 21)
    for (k0, d0), (k1, d1) in zip(res, unpack_packed(buf)):
        assert np.array_equal(k0, k1) and np.array_equal(d0, d1)


def test_gloo_two_rank_c4_gather_matches_single_process():
    tag, got, sizes = _run(_c4_worker)
    from orb_slam2_2021_amd import synth_frame
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    assert len(got) == N_FRAMES
    for i, (kb, db) in enumerate(got):
        k, d = ref(synth_frame(i, ROWS, COLS))
        assert kb == k.tobytes() and db == d.tobytes()
    # only used bytes crossed: each payload is exactly its packed size
    for r in range(2):
        n = [len(RefExtractor(500, 1.2, 4, 20, 7)(synth_frame(i, ROWS, COLS))[0])
             for i in shard_frames(N_FRAMES, 2, r)]
        assert sizes[r] == packed_bytes(len(n), sum(n))


def test_gloo_two_rank_c4_fixed_count_gather():
    tag, got, _ = _run(_c4_fixed_worker)
    from orb_slam2_2021_amd import synth_frame
    from oracle.orbref import RefExtractor
    ref = RefExtractor(500, 1.2, 4, 20, 7)
    assert len(got) == N_FRAMES
    for i, (kb, db) in enumerate(got):
        k, d = ref(synth_frame(i, ROWS, COLS))
        assert kb == k.tobytes() and db == d.tobytes()


def test_gloo_two_rank_c5_replicated_map_sharded_frames():
    from oracle import orbref
    tag, rows, n_frames = _run(_c5_worker)
    G, frames = _c5_scene()
    rows = np.frombuffer(rows, np.int32)
    m = len(G.flags)
    rows = rows.reshape(n_frames, 3 + m)
    for i in range(n_frames):
        nm, best, nv, _ = orbref.search_local_points(frames[i], G, 0.1823215568, 3.0, 0.8)
        assert rows[i, 0] == i and rows[i, 1] == nm and rows[i, 2] == nv
        assert np.array_equal(rows[i, 3:], best)
    assert rows[:, 1].sum() > 0


def test_bench_spawns_torchrun_for_n_gpus(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    cmd, env = calls[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_rank_refuses_world_mismatch(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=2" in str(e.value.code)


def test_rccl_binding_resolves_the_p2p_api():
    """The C4 transfer binding (orb_slam2_2021_amd.rccl) finds torch's librccl and every entry it
    calls, without touching a GPU."""
    from orb_slam2_2021_amd import rccl
    lib = rccl.lib()
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclSend", "ncclRecv", "ncclGroupStart",
              "ncclGroupEnd", "ncclCommDestroy", "ncclGetErrorString"):
        assert getattr(lib, f) is not None
    assert lib.ncclGetErrorString(0)
