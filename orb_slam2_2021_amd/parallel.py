"""Frame sharding and the exchange steps across GPUs (one process per GPU, torch.distributed).

Extraction is independent per image (ORBextractor::operator(), ORBextractor.cc:1041-1103) and
SearchForTriangulation per KeyFrame pair, so frames shard embarrassingly: rank r owns a block of
frames and no collective touches the data path. The exchange steps BASELINE.json names:

* C4: every rank's keypoints and descriptors gathered to rank 0. Each rank packs its used slots
  on the device (orbfe_pack_keypoints_device, include/orbfe_pack.h: a header of per-image counts,
  then the keypoints and descriptors back to back), and rank 0 receives each payload
  point-to-point over RCCL (xGMI: one link per peer). gather_fixed moves a fixed byte count
  (the packed worst case, about 1 % above a full batch's used bytes), so no size crosses to the
  host and the exchange never synchronises it; gather_packed exchanges the sizes first and moves
  exactly the used bytes (one host sync per call).
* C5: the local map (the MapPoint SoA Tracking::SearchLocalPoints projects, Tracking.cc:1164-1216)
  is replicated: broadcast once from rank 0, then every rank matches its own frames against it.
"""
from __future__ import annotations

from ctypes import c_size_t, c_void_p
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import KEYPOINT_DTYPE


def shard_frames(n_frames: int, world: int, rank: int) -> range:
    """Contiguous block of frame indices owned by `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


# ---- the packed form of a batch's keypoints + descriptors (include/orbfe_pack.h) ----

def _align16(x: int) -> int:
    return (x + 15) & ~15


def packed_bytes(n_images: int, total_keypoints: int) -> int:
    head = _align16(4 * (1 + n_images))
    return _align16(head + 28 * total_keypoints) + 32 * total_keypoints


def pack_host(results: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]]) -> np.ndarray:
    """Host-side packing in the device layout (for CPU ranks and tests)."""
    counts = np.array([len(k) for k, _ in results], np.int32)
    total = int(counts.sum())
    out = np.zeros(packed_bytes(len(results), total), np.uint8)
    head = _align16(4 * (1 + len(results)))
    out[:4] = np.frombuffer(np.int32(len(results)).tobytes(), np.uint8)
    out[4:4 + 4 * len(results)] = np.frombuffer(counts.tobytes(), np.uint8)
    kp = np.concatenate([np.ascontiguousarray(k, KEYPOINT_DTYPE) for k, _ in results]) if total else \
        np.zeros(0, KEYPOINT_DTYPE)
    out[head:head + 28 * total] = np.frombuffer(kp.tobytes(), np.uint8)
    doff = _align16(head + 28 * total)
    for (k, d) in results:
        if len(k):
            n = len(k)
            out[doff:doff + 32 * n] = np.ascontiguousarray(d, np.uint8).reshape(-1)
            doff += 32 * n
    return out


def unpack_packed(buf: np.ndarray) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Per-image (keypoints, descriptors) from a packed buffer."""
    buf = np.ascontiguousarray(buf, np.uint8)
    n_img = int(np.frombuffer(buf[:4].tobytes(), np.int32)[0])
    counts = np.frombuffer(buf[4:4 + 4 * n_img].tobytes(), np.int32)
    total = int(counts.sum())
    head = _align16(4 * (1 + n_img))
    kp = np.frombuffer(buf[head:head + 28 * total].tobytes(), KEYPOINT_DTYPE)
    doff = _align16(head + 28 * total)
    de = buf[doff:doff + 32 * total].reshape(total, 32)
    out, o = [], 0
    for c in counts:
        out.append((kp[o:o + c].copy(), de[o:o + c].copy()))
        o += int(c)
    return out


def pack_keypoints_device(n_images: int, d_counts: int, d_kps: int, d_desc: int, cap: int,
                          d_out: int, out_cap: int, d_total: int, stream: int = 0) -> None:
    """orbfe_pack_keypoints_device: async on `stream`; the size lands in the int64 at d_total."""
    L.check(L.lib().orbfe_pack_keypoints_device(int(n_images), c_void_p(d_counts), c_void_p(d_kps),
                                                c_void_p(d_desc), int(cap), c_void_p(d_out),
                                                c_size_t(out_cap), c_void_p(d_total), c_void_p(stream)),
            "orbfe_pack_keypoints_device")


def gather_packed(payload, size, dst: int = 0, recv: Optional[Sequence] = None):
    """Gather every rank's packed payload to `dst`: sizes first (all_gather of one int64 per
    rank), then one point-to-point transfer per peer of exactly its used bytes.

    payload: uint8 tensor holding this rank's packed batch; size: int64 tensor [1] with its byte
    count (on the payload's device: written by the pack kernel, or set by the host).
    recv: on dst, per-rank uint8 receive buffers (allocated if None).
    Returns (list of per-rank uint8 tensors of exact size on dst / None elsewhere, sizes).
    Works on any backend: RCCL ("nccl") on GPUs, gloo on CPU tensors."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = [torch.empty(1, dtype=torch.int64, device=size.device) for _ in range(world)]
    dist.all_gather(sizes, size.reshape(1))
    sizes_h = [int(x) for x in torch.cat(sizes).cpu().tolist()]
    ops = []
    out = None
    if rank == dst:
        out = []
        for r in range(world):
            if r == dst:
                out.append(payload[:sizes_h[r]])
                continue
            buf = recv[r] if recv is not None else torch.empty(sizes_h[r], dtype=torch.uint8,
                                                               device=payload.device)
            if buf.numel() < sizes_h[r]:
                raise ValueError(f"receive buffer for rank {r} too small")
            out.append(buf[:sizes_h[r]])
            ops.append(dist.P2POp(dist.irecv, out[-1], r))
    else:
        ops.append(dist.P2POp(dist.isend, payload[:sizes_h[rank]], dst))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out, sizes_h


def gather_fixed(payload, nbytes: int, dst: int = 0, recv: Optional[Sequence] = None):
    """Gather the first `nbytes` of every rank's payload to `dst` with point-to-point transfers
    and no size exchange: the packed header (n_images, counts) tells the receiver what is used.
    Enqueued on the caller's current stream; the host never waits for the device (the returned
    requests are already waited on the stream, which is what torch's NCCL work.wait() does).

    recv: on dst, per-rank uint8 buffers of at least nbytes (allocated if None). Returns the list
    of per-rank views on dst (dst's own entry is payload[:nbytes]) and None elsewhere. The views
    alias `payload` / `recv`: valid until the caller reuses them."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if payload.numel() < nbytes:
        raise ValueError("payload smaller than nbytes")
    ops, out = [], None
    if rank == dst:
        out = []
        for r in range(world):
            if r == dst:
                out.append(payload[:nbytes])
                continue
            buf = recv[r] if recv is not None else torch.empty(nbytes, dtype=torch.uint8, device=payload.device)
            if buf.numel() < nbytes:
                raise ValueError(f"receive buffer for rank {r} too small")
            out.append(buf[:nbytes])
            ops.append(dist.P2POp(dist.irecv, out[-1], r))
    else:
        ops.append(dist.P2POp(dist.isend, payload[:nbytes], dst))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return out


def packed_size(buf) -> int:
    """Used bytes of a packed buffer (numpy or a uint8 tensor), from its header."""
    a = np.ascontiguousarray(buf[:4].cpu().numpy() if hasattr(buf, "cpu") else buf[:4], np.uint8)
    n_img = int(a.view(np.int32)[0])
    h = buf[4:4 + 4 * n_img]
    c = np.ascontiguousarray(h.cpu().numpy() if hasattr(h, "cpu") else h, np.uint8).view(np.int32)
    return packed_bytes(n_img, int(c.astype(np.int64).sum()))


def broadcast_arrays(arrays: Dict[str, np.ndarray], device, src: int = 0) -> Dict[str, object]:
    """C5's replicated local map: the MapPoint SoA (names -> numpy arrays, meaningful on `src`;
    the other ranks pass arrays of the same shapes and dtypes) broadcast from `src` into tensors on
    every rank's `device`. Returns {name: tensor}."""
    import torch
    import torch.distributed as dist
    out = {}
    for name in sorted(arrays):
        a = np.ascontiguousarray(arrays[name])
        t = torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(device)
        dist.broadcast(t, src=src)
        out[name] = t
    return out
