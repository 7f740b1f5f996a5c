"""Multi-GPU CombineCC through the C ABI (include/gsgpu.h gs_comm_* / gs_cc_merge_window, csrc/comm.hip).

``Comm`` wraps one rank's RCCL communicator; ``DisjointSet.merge_window(comm, mode)`` exchanges
the window's partial summary and closes the window — the windowAll gather
(SummaryBulkAggregation.java:81-83), ConnectedComponentsTree's pairwise rounds
(SummaryTreeReduce.java:95-123), or the replicated all-gather (bench default). The unique id is
made by rank 0 and handed to every rank by torch.distributed (any side channel works: a Java host
would put it in the job configuration).
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

from . import _abi
from ._abi import GS_MERGE_ALLGATHER, GS_MERGE_GATHER, GS_MERGE_PREFILTER, GS_MERGE_TREE, call

MODES = {"allgather": GS_MERGE_ALLGATHER, "gather": GS_MERGE_GATHER, "tree": GS_MERGE_TREE,
         "prefilter": GS_MERGE_PREFILTER}   # prefilter: fold_windows only
UNIQUE_ID_BYTES = 128


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    call("gs_comm_unique_id", buf, UNIQUE_ID_BYTES)
    return buf.raw


class Comm:
    """One rank's communicator (RCCL over xGMI), or one member of an in-process group (local)."""

    def __init__(self, handle: ctypes.c_void_p, device: int):
        self._h = handle
        self.device = device

    @classmethod
    def create(cls, uid: bytes, rank: int, world: int, device: int) -> "Comm":
        """gs_comm_create: every rank calls this concurrently (ncclCommInitRank is collective)."""
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), UNIQUE_ID_BYTES)
        call("gs_comm_create", ctypes.byref(h), buf, int(rank), int(world), int(device))
        return cls(h, device)

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "Comm":
        """Rank 0 makes the unique id, torch.distributed broadcasts it, every rank joins."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
        return cls.create(obj[0], rank, world, device)

    @classmethod
    def local_group(cls, world: int, device: int = 0) -> List["Comm"]:
        """gs_comm_create_local: `world` communicators in this process on one device (drive each
        rank from its own thread; tests of the exchange where RCCL cannot run several ranks)."""
        arr = (ctypes.c_void_p * world)()
        call("gs_comm_create_local", arr, int(world), int(device))
        return [cls(ctypes.c_void_p(arr[r]), device) for r in range(world)]

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise RuntimeError("Comm is closed")
        return self._h

    def info(self) -> Tuple[int, int, int, int, int, int]:
        """(rank, world, bytes_sent, bytes_recv, exchanges, overflows): overflows = speculative
        all-gather rounds a delta outgrew (each followed by one exact round)."""
        r, w = ctypes.c_int(), ctypes.c_int()
        s, v, e, o = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        call("gs_comm_info", self.handle, ctypes.byref(r), ctypes.byref(w), ctypes.byref(s), ctypes.byref(v),
             ctypes.byref(e), ctypes.byref(o))
        return r.value, w.value, s.value, v.value, e.value, o.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            _abi.lib().gs_comm_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass
