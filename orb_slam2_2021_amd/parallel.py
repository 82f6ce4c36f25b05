"""Frame sharding and result gathering across GPUs (one process per GPU, torch.distributed).

Extraction is independent per image (ORBextractor::operator(), ORBextractor.cc:1041-1103) and
SearchForTriangulation per KeyFrame pair, so frames shard embarrassingly: rank r owns a
contiguous block of frames and no collective touches the data path. The one exchange step the
north star names -- gathering every rank's keypoints and descriptors to rank 0 (BASELINE config
C4) -- is a fixed-capacity gather of (counts, keypoints, descriptors) buffers over RCCL (xGMI),
unpacked into per-frame results on the destination.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import KEYPOINT_DTYPE


def shard_frames(n_frames: int, world: int, rank: int) -> range:
    """Contiguous block of frame indices owned by `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_to_root(counts, kps_bytes, desc_bytes, dst: int = 0):
    """Gather fixed-capacity per-image buffers of every rank to `dst`.

    counts: int32 tensor [n_img]; kps_bytes / desc_bytes: uint8 tensors [n_img * cap * 28 / 32].
    Returns lists of per-rank tensors on `dst` (None elsewhere). Works on any backend: RCCL
    ("nccl") on GPUs, gloo on CPU tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rank = dist.get_rank()
    out = None
    if rank == dst:
        out = ([torch.empty_like(counts) for _ in range(world)],
               [torch.empty_like(kps_bytes) for _ in range(world)],
               [torch.empty_like(desc_bytes) for _ in range(world)])
    dist.gather(counts, out[0] if out else None, dst=dst)
    dist.gather(kps_bytes, out[1] if out else None, dst=dst)
    dist.gather(desc_bytes, out[2] if out else None, dst=dst)
    return out


def unpack(counts: np.ndarray, kps_bytes: np.ndarray, desc_bytes: np.ndarray,
           cap: int) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Per-image (keypoints, descriptors) from fixed-capacity buffers."""
    n_img = len(counts)
    kp = np.frombuffer(np.ascontiguousarray(kps_bytes).tobytes(), KEYPOINT_DTYPE).reshape(n_img, cap)
    de = np.ascontiguousarray(desc_bytes).reshape(n_img, cap, 32)
    return [(kp[i, :counts[i]].copy(), de[i, :counts[i]].copy()) for i in range(n_img)]


def pack(results: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]], cap: int):
    """Inverse of unpack: fixed-capacity (counts, keypoint bytes, descriptor bytes)."""
    n_img = len(results)
    counts = np.zeros(n_img, np.int32)
    kp = np.zeros((n_img, cap), KEYPOINT_DTYPE)
    de = np.zeros((n_img, cap, 32), np.uint8)
    for i, (k, d) in enumerate(results):
        n = len(k)
        if n > cap:
            raise ValueError("capacity exceeded")
        counts[i] = n
        kp[i, :n] = k
        if n:
            de[i, :n] = d
    return counts, np.frombuffer(kp.tobytes(), np.uint8).copy(), de.reshape(-1).copy()
