"""Multi-GPU CombineCC: log2(P) pairwise tree merge of per-rank partial summaries.

Restates the reference's tree reduction ``SummaryTreeReduce.enhance``
(src/main/java/org/apache/flink/graph/streaming/SummaryTreeReduce.java:95-123: each round keys
partial summaries by ``partition / 2`` so pairs of partitions meet at one subtask and are
combined with CombineCC, until one remains for the ``windowAll`` reduce and the Merger,
SummaryAggregation.java:106-119) as point-to-point transfers between GPU ranks over
``torch.distributed`` (backend ``nccl`` = RCCL over xGMI on MI355X; ``gloo`` for CPU tests).

One process per GPU; every rank keeps its own cumulative summary of the edges it folded (plus
what it received). Per window, a rank's partial summary is the set of (vertex, parent) pairs it
gained that window (``DisjointSet.export_marks``: roots it hooked, self-loop singletons), i.e.
exactly the connectivity the rank has and rank 0 may not. Round r (step = 2^r): rank
i + step sends its pairs to rank i (i % 2^(r+1) == 0), which folds them in
(``DisjointSet.merge`` semantics = union over the pairs), marking what it gains, and forwards
that in a later round. After ceil(log2 P) rounds rank 0 holds the union of all ranks' edges;
it closes the window (compression = canonical emission). Only rank 0 emits.

The summary object needs: ``export_marks(buf_int32_tensor) -> n``, ``fold_pairs(buf, n,
id_bits=32)``, ``close_window()`` — gsgpu.DisjointSet on GPU ranks; the tests plug a CPU
summary with the same three methods to run the exchange under gloo.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist


def tree_schedule(rank: int, world: int) -> List[Tuple[str, int]]:
    """[(role, peer)] per round for this rank: ('send', dst) / ('recv', src) / ('idle', -1)."""
    out = []
    step = 1
    while step < world:
        if rank % (2 * step) == step:
            out.append(("send", rank - step))
        elif rank % (2 * step) == 0 and rank + step < world:
            out.append(("recv", rank + step))
        else:
            out.append(("idle", -1))
        step *= 2
    return out


class TreeMerge:
    def __init__(self, summary, capacity_pairs: int, device: torch.device, group=None):
        self.summary = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        self.schedule = tree_schedule(self.rank, self.world)
        self.cap = int(capacity_pairs)
        needs_buf = any(r != "idle" for r, _ in self.schedule)
        self.buf = torch.empty(2 * self.cap if needs_buf else 2, dtype=torch.int32, device=device)
        self.cnt = torch.zeros(1, dtype=torch.int64, device=device)
        # gloo moves host tensors only: stage device buffers through pinned host copies (tests
        # of the multi-rank path on one GPU); nccl (RCCL) sends device memory directly
        self.stage = (dist.get_backend(group) == "gloo" and torch.device(device).type == "cuda")
        if self.stage:
            self.hbuf = torch.empty(self.buf.numel(), dtype=torch.int32).pin_memory()
            self.hcnt = torch.zeros(1, dtype=torch.int64)
        self.bytes_sent = 0
        self.bytes_recv = 0

    def _grank(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _send(self, n: int, dst: int) -> None:
        if self.stage:
            self.hcnt.fill_(n)
            dist.send(self.hcnt, dst, group=self.group)
            if n:
                self.hbuf[: 2 * n].copy_(self.buf[: 2 * n])
                dist.send(self.hbuf[: 2 * n], dst, group=self.group)
            return
        self.cnt.fill_(n)
        dist.send(self.cnt, dst, group=self.group)
        if n:
            dist.send(self.buf[: 2 * n], dst, group=self.group)

    def _recv(self, src: int) -> int:
        c = self.hcnt if self.stage else self.cnt
        dist.recv(c, src, group=self.group)
        n = int(c.item())
        if n > self.cap:
            raise RuntimeError("partial summary of %d pairs exceeds capacity %d" % (n, self.cap))
        if n:
            if self.stage:
                dist.recv(self.hbuf[: 2 * n], src, group=self.group)
                self.buf[: 2 * n].copy_(self.hbuf[: 2 * n])
            else:
                dist.recv(self.buf[: 2 * n], src, group=self.group)
        return n

    def merge_window(self) -> bool:
        """Exchange this window's partial summaries; returns True on rank 0 (which emitted)."""
        for role, peer in self.schedule:
            if role == "send":
                n = self.summary.export_marks(self.buf, self.cap)
                self._send(n, self._grank(peer))
                self.bytes_sent += 8 * n
                break                                   # a sender is done for this window
            if role == "recv":
                n = self._recv(self._grank(peer))
                if n:
                    self.summary.fold_pairs(self.buf, n, id_bits=32)
                self.bytes_recv += 8 * n
        # every rank closes its window: rank 0's close is the Merger's emission; on the other
        # ranks it keeps their own giant-component filter current for their next fold
        self.summary.close_window()
        return self.rank == 0
