"""C4's device side (BASELINE config C4: frames sharded over GPUs, keypoints + descriptors
gathered to rank 0; per-frame independence of ORBextractor::operator(), ORBextractor.cc:1041-1103):

* the device packer k_pack (orbfe_pack_keypoints_device) against the host packer pack_host, byte
  for byte over the whole used length -- header, zero padding, keypoints, descriptors -- for
  counts 0, 1 and cap, and for the bench's own 64-image C3 extraction;
* bench.py's Gatherer path with two ranks on GPU 0 over gloo (`--rehearse --gpus 2`): rank 0's
  received payloads, unpacked, equal what each rank extracted, bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

from orb_slam2_2021_amd import KEYPOINT_DTYPE, ORBextractor, synth_frame
from orb_slam2_2021_amd.parallel import (pack_host, pack_keypoints_device, packed_bytes, packed_size,
                                         unpack_packed)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_pack(counts, kps, desc, cap, fill=0xAB):
    """Pack on the device; the output buffer starts as `fill` garbage so that unwritten padding
    shows. Returns (packed bytes up to the reported size, reported size)."""
    import torch
    n = len(counts)
    cap_bytes = packed_bytes(n, n * cap)
    d_cnt = torch.from_numpy(np.asarray(counts, np.int32)).cuda()
    d_kps = torch.from_numpy(kps.view(np.uint8).reshape(-1).copy()).cuda()
    d_desc = torch.from_numpy(desc.reshape(-1).copy()).cuda()
    out = torch.full((cap_bytes + 64,), fill, dtype=torch.uint8, device="cuda")
    tot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    pack_keypoints_device(n, d_cnt.data_ptr(), d_kps.data_ptr(), d_desc.data_ptr(), cap, out.data_ptr(),
                          cap_bytes, tot.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    size = int(tot.item())
    return out.cpu().numpy(), size


def _random_batch(rng, counts, cap):
    n = len(counts)
    kps = np.frombuffer(rng.integers(0, 256, n * cap * 28, dtype=np.uint8).tobytes(), KEYPOINT_DTYPE).copy()
    desc = rng.integers(0, 256, (n * cap, 32), dtype=np.uint8)
    return kps, desc


@pytest.mark.parametrize("counts", [[0, 1, 64, 0, 17], [0], [1], [64], [64] * 9, [0] * 5, [3, 0, 0, 5, 64, 1, 2]])
def test_k_pack_equals_pack_host(require_gpu, counts):
    cap = 64
    rng = np.random.default_rng(len(counts) * 131 + sum(counts))
    kps, desc = _random_batch(rng, counts, cap)
    res = [(kps[i * cap:i * cap + c], desc[i * cap:i * cap + c]) for i, c in enumerate(counts)]
    want = pack_host(res)
    got, size = _device_pack(counts, kps, desc, cap)
    assert size == len(want) == packed_bytes(len(counts), sum(counts))
    assert np.array_equal(got[:size], want), np.flatnonzero(got[:size] != want)[:10]
    assert packed_size(got) == size
    for (k0, d0), (k1, d1) in zip(res, unpack_packed(got[:size])):
        assert k0.tobytes() == k1.tobytes() and np.array_equal(d0, d1)


def test_k_pack_clamps_counts_to_cap(require_gpu):
    """A count above cap (or below 0) packs as cap (0), as the kernel documents."""
    cap = 16
    rng = np.random.default_rng(3)
    kps, desc = _random_batch(rng, [0, 0, 0], cap)
    got, size = _device_pack([20, -4, 5], kps, desc, cap)
    want = pack_host([(kps[:16], desc[:16]), (kps[:0], desc[:0]), (kps[32:37], desc[32:37])])
    assert size == len(want) and np.array_equal(got[:size], want)


def test_k_pack_bench_c3_batch(require_gpu):
    """The bench's 64-image C3 extraction (extract_batch_device output, cap-slot rows) packed on
    the device equals pack_host of the same outputs copied to the host."""
    import torch
    B, H, W = 32, 376, 1241
    imgs = np.zeros((2 * B, H, W), np.uint8)
    for i in range(B):
        imgs[i], imgs[B + i] = synth_frame(i, H, W, right=True)
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    cap = ext.max_keypoints(H, W)
    d_img = torch.from_numpy(imgs).cuda()
    kps = torch.empty(2 * B * cap * 28, dtype=torch.uint8, device="cuda")
    desc = torch.empty(2 * B * cap * 32, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()  # one explicit stream orders extraction -> pack (0 = the handle's own)
    ext.extract_batch_device(2 * B, d_img.data_ptr(), H * W, H, W, W, kps.data_ptr(), desc.data_ptr(), cap,
                             cnt.data_ptr(), stream=s.cuda_stream)
    cap_bytes = packed_bytes(2 * B, 2 * B * cap)
    out = torch.full((cap_bytes,), 0xCD, dtype=torch.uint8, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    pack_keypoints_device(2 * B, cnt.data_ptr(), kps.data_ptr(), desc.data_ptr(), cap, out.data_ptr(), cap_bytes,
                          tot.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    K = kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(2 * B, cap)
    D = desc.cpu().numpy().reshape(2 * B, cap, 32)
    C = cnt.cpu().numpy()
    want = pack_host([(K[i, :C[i]], D[i, :C[i]]) for i in range(2 * B)])
    size = int(tot.item())
    assert size == len(want)
    assert np.array_equal(out.cpu().numpy()[:size], want)
    assert C.min() >= 2000
    # the fixed-count transfer's overhead: the worst case is within 2 % of the used bytes
    assert cap_bytes <= 1.02 * size


@pytest.mark.parametrize("root_share", ["-1", "0.5"])
def test_bench_gatherer_two_ranks_on_one_gpu(require_gpu, tmp_path, root_share):
    """bench.py --rehearse --gpus 2: two ranks on GPU 0 over gloo run the bench's whole multi-rank
    orchestration (Gatherer: device pack on the matching stream, fixed-count point-to-point
    transfers to rank 0). Rank 0's received payloads must equal each rank's own extraction of its
    last sub-batch, bit for bit. --root-share 0.5: rank 0 extracts on every other slot only and
    receives the peer's payload on the others (receive-only gathers), so the ranks' exchanges
    still pair up slot by slot."""
    d = str(tmp_path / "gather")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--rehearse", "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--batches-per-step", "4", "--input-batches", "2", "--probe-subbatches", "2",
           "--no-cpu", "--no-legs", "--no-parity", "--dump-gather", d, "--root-share", root_share]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for rank in range(2):
        own = np.load(os.path.join(d, f"{rank}_own.npz"))
        buf = np.fromfile(os.path.join(d, f"{rank}_gathered.bin"), np.uint8)
        size = packed_size(buf)
        counts = own["counts"]
        assert size == packed_bytes(len(counts), int(counts.sum()))
        got = unpack_packed(buf[:size])
        assert [len(k) for k, _ in got] == list(counts)
        assert np.concatenate([k for k, _ in got]).tobytes() == own["kps"].tobytes()
        assert np.concatenate([x for _, x in got]).reshape(-1).tobytes() == own["desc"].tobytes()
        assert counts.min() >= 2000
    # the two ranks extracted different frames (frame sharding)
    a = np.load(os.path.join(d, "0_own.npz"))["desc"]
    b = np.load(os.path.join(d, "1_own.npz"))["desc"]
    assert a.tobytes() != b.tobytes()


def test_rccl_self_transfers_on_a_stream(require_gpu):
    """orb_slam2_2021_amd.rccl on a world-1 communicator: send / receive pairs with itself on a
    caller's stream (the one-GPU proxy of C4's root) move the bytes exactly, ordered by the stream
    alone (the payload is written on the same stream right before)."""
    import torch
    from orb_slam2_2021_amd.rccl import RcclComm, unique_id
    comm = RcclComm(1, 0, unique_id())
    try:
        s = torch.cuda.Stream()
        n = 7_772_432 + 13
        src = torch.empty(n, dtype=torch.uint8, device="cuda")
        dst = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
        with torch.cuda.stream(s):
            src.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda"))
        comm.self_copies([src.data_ptr()], n, [[d.data_ptr() for d in dst]], s.cuda_stream)
        s.synchronize()
        for d in dst:
            assert torch.equal(d, src)
    finally:
        comm.close()
