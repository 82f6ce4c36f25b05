"""C4's transfers as RCCL point-to-point calls on a caller's stream.

torch.distributed's NCCL process group runs every collective on a stream of its own and orders it
after the caller's stream with an event wait. On MI355X, an otherwise idle stream made to wait on
the matching stream's pending event once per sub-batch measured 52.7k instead of 83.3k stereo
frames/s on one GPU (`--gather-proxy 2`, wait-only mode), while the same
transfers enqueued on the matching stream itself cost 2 %. This module calls RCCL's C API (the
librccl.so torch already loaded, so one RCCL instance per process) with the matching stream as the
launch stream: ncclSend / ncclRecv in one group per sub-batch, ordered after the pack kernel by the
stream itself, no event. The communicator is built once from a unique id that rank 0 creates and
torch.distributed broadcasts.

A world-1 communicator sending to and receiving from itself moves the same bytes through the same
RCCL kernels on one GPU: `bench.py --gather-proxy N` uses that (N - 1 self transfers per sub-batch)
and tests/test_gpu_gather.py checks the bytes.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_int, c_size_t, c_void_p
from typing import Optional, Sequence

NCCL_UINT8 = 1  # ncclUint8 (nccl.h: ncclInt8 = 0, ncclUint8 = 1)


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_uint8 * 128)]  # NCCL_UNIQUE_ID_BYTES


_LIB = None


def lib():
    """torch's librccl.so (already loaded by torch: the same library instance)."""
    global _LIB
    if _LIB is None:
        import torch
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        l = ctypes.CDLL(path)
        l.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        l.ncclCommInitRank.argtypes = [ctypes.POINTER(c_void_p), c_int, _UniqueId, c_int]
        l.ncclSend.argtypes = [c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]
        l.ncclRecv.argtypes = [c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]
        l.ncclGroupStart.argtypes = []
        l.ncclGroupEnd.argtypes = []
        l.ncclCommDestroy.argtypes = [c_void_p]
        l.ncclGetErrorString.argtypes = [c_int]
        l.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclSend", "ncclRecv", "ncclGroupStart",
                  "ncclGroupEnd", "ncclCommDestroy"):
            getattr(l, f).restype = c_int
        _LIB = l
    return _LIB


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ncclGetErrorString(rc)
        raise RuntimeError(f"{what}: {msg.decode() if msg else 'error'} (ncclResult {rc})")


def unique_id() -> bytes:
    uid = _UniqueId()
    _check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return bytes(uid.internal)


class RcclComm:
    """One RCCL communicator over `nranks` processes (one GPU each; the caller's current HIP
    device must be its GPU). `uid` is rank 0's unique_id(), the same bytes on every rank."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != 128:
            raise ValueError("an RCCL unique id is 128 bytes")
        u = _UniqueId()
        ctypes.memmove(u.internal, uid, 128)
        self._comm = c_void_p()
        _check(lib().ncclCommInitRank(ctypes.byref(self._comm), int(nranks), u, int(rank)), "ncclCommInitRank")
        self.nranks, self.rank = int(nranks), int(rank)

    @classmethod
    def from_process_group(cls) -> "RcclComm":
        """All ranks of the default torch.distributed group; rank 0's unique id is broadcast over
        it (once, outside any timed region)."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(), dist.get_rank()
        box = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return cls(world, rank, box[0])

    def gather(self, send_ptrs: Sequence[int], nbytes: int, recv_ptrs: Optional[Sequence[Sequence[int]]],
               root: int, stream: int) -> None:
        """Every rank's payloads to `root`, one RCCL group on `stream` (a hipStream_t address),
        ordered by the stream alone: send_ptrs[j] holds this rank's j-th payload (its first
        `nbytes`); on the root, rank r's j-th payload lands at recv_ptrs[j][r] (the root's own
        entries are ignored: its payloads stay where they are)."""
        l, c, s = lib(), self._comm, c_void_p(stream)
        _check(l.ncclGroupStart(), "ncclGroupStart")
        try:
            for j, sp in enumerate(send_ptrs):
                if self.rank == root:
                    for r in range(self.nranks):
                        if r != root:
                            _check(l.ncclRecv(c_void_p(recv_ptrs[j][r]), nbytes, NCCL_UINT8, r, c, s), "ncclRecv")
                else:
                    _check(l.ncclSend(c_void_p(sp), nbytes, NCCL_UINT8, root, c, s), "ncclSend")
        finally:
            _check(l.ncclGroupEnd(), "ncclGroupEnd")

    def self_copies(self, send_ptrs: Sequence[int], nbytes: int, recv_ptrs: Sequence[Sequence[int]],
                    stream: int) -> None:
        """For payload j (send_ptrs[j]), one send / receive pair of this rank with itself into each
        of recv_ptrs[j], all in one group (the one-GPU proxy of a root receiving from that many
        peers)."""
        l, c, s = lib(), self._comm, c_void_p(stream)
        _check(l.ncclGroupStart(), "ncclGroupStart")
        try:
            for sp, rp in zip(send_ptrs, recv_ptrs):
                for p in rp:
                    _check(l.ncclSend(c_void_p(sp), nbytes, NCCL_UINT8, self.rank, c, s), "ncclSend")
                    _check(l.ncclRecv(c_void_p(p), nbytes, NCCL_UINT8, self.rank, c, s), "ncclRecv")
        finally:
            _check(l.ncclGroupEnd(), "ncclGroupEnd")

    def close(self) -> None:
        if self._comm:
            lib().ncclCommDestroy(self._comm)
            self._comm = c_void_p()
