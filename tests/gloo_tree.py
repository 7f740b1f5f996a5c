"""TEST MODEL (not the product): the multi-GPU CombineCC exchanges restated over torch.distributed,
so the exchange logic runs multi-process under gloo on CPU (tests/test_tree_gloo.py) and bench.py's
--dist-backend gloo test mode can put several ranks on one GPU. The product exchange is
gelly-streaming_amd/csrc/comm.hip (gs_cc_merge_window over RCCL), the same three modes with the same
delta contract.

Three exchanges behind one contract (``merge_window()`` after each window's fold; True on the
rank that emitted):

``AllgatherMerge`` (bench.py's gloo-mode default): replicated summaries. Every rank keeps the GLOBAL summary: per
window each rank exports its delta (the connectivity its own slice added), the deltas are
all-gathered (one RCCL all-gather of slots padded to the largest delta; on xGMI every pair of
GPUs has its own link), and each rank folds the others' deltas with marking paused. Every rank's filter is then the global giant component, so the
deltas shrink to the genuinely new connectivity (RMAT-26, 8 ranks, window 64: 14K pairs per rank
instead of 132K) and every rank's fold is as fast as a single GPU's (tools/sim_ranks.py).
``GatherMerge``: the reference's windowAll reduce (SummaryBulkAggregation.java:81: every
partition's partial summary goes to the one parallelism-1 task) as one flat gather to rank 0 —
every other rank sends its window's pairs straight to rank 0 over its own xGMI link, all at once,
and rank 0 folds them.
``TreeMerge`` (ConnectedComponentsTree): log2(P) pairwise rounds (SummaryTreeReduce.enhance).
``PrefilterMerge`` (GS_MERGE_PREFILTER, bench.py's default over RCCL at P > 1): ranks 1..P-1 filter
their slices against rank 0's broadcast giant bitmap and send the survivors to rank 0 (CPU tests
only: the product path is comm.hip).

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

import numpy as np
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
        # an export holds at most 2 x capacity pairs (a vertex's self-loop first touch and its hook:
        # include/gsgpu.h gs_cc_export_marks_async)
        self.cap = 2 * int(capacity_pairs)
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


class GatherMerge:
    """Flat gather of every rank's window pairs to rank 0 (windowAll reduce + Merger).

    Per window, rank r != 0: export its marks into one of two device buffers (alternating, so
    a send still in flight is never overwritten: the buffer's previous sends are waited on, on
    the current stream, before the next export into it) and isend the count and the pairs to
    rank 0. Rank 0 posts the count receives before its own fold is enqueued, learns the counts
    (one host sync), receives every payload into one contiguous buffer (all peers at once, on a
    side stream so the transfers overlap its fold), and folds all pairs in one launch; then every
    rank closes its window. Senders never wait for rank 0's emission: they run at most two
    windows ahead. Summary contract as TreeMerge.
    """

    def __init__(self, summary, capacity_pairs: int, device: torch.device, group=None):
        self.summary = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        # an export holds at most 2 x capacity pairs; rank 0 receives up to (P - 1) exports
        self.cap = 2 * int(capacity_pairs)
        self.total_cap = self.cap * max(self.world - 1, 1)
        self.stage = (dist.get_backend(group) == "gloo" and self.device.type == "cuda")
        if self.rank == 0:
            self.cnts = torch.zeros(max(self.world - 1, 1), dtype=torch.int64,
                                    device="cpu" if self.stage else self.device)
            self.buf = torch.empty(2 * max(self.cap, 1), dtype=torch.int32, device=self.device)   # grows
            self.hbuf = torch.empty(0, dtype=torch.int32).pin_memory() if self.stage else None
            self.side = torch.cuda.Stream(self.device) if self.device.type == "cuda" and not self.stage else None
            self.free_ev = None            # recorded after the last fold out of self.buf
            self._cnt_works = None
        else:
            self.bufs = [torch.empty(2 * self.cap, dtype=torch.int32, device=self.device) for _ in range(2)]
            self.cnt = [torch.zeros(1, dtype=torch.int64, device="cpu" if self.stage else self.device) for _ in range(2)]
            self.hbufs = [torch.empty(2 * self.cap, dtype=torch.int32).pin_memory() for _ in range(2)] if self.stage else None
            self.works = [[], []]
            self.turn = 0
        self.bytes_sent = 0
        self.bytes_recv = 0
        dist.barrier(group=self.group)     # communicators up before the first point-to-point batch

    def _grank(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def before_fold(self) -> None:
        """Rank 0: post this window's count receives before its own fold is enqueued, so the
        counts are not ordered behind the fold on the communicator's stream."""
        if self.rank != 0 or self.world == 1 or self._cnt_works is not None:
            return
        ops = [dist.P2POp(dist.irecv, self.cnts[i - 1:i], self._grank(i), group=self.group)
               for i in range(1, self.world)]
        self._cnt_works = dist.batch_isend_irecv(ops)

    def merge_window(self) -> bool:
        if self.world == 1:
            self.summary.close_window()
            return True
        if self.rank != 0:
            t = self.turn
            for w in self.works[t]:                    # the previous sends out of this buffer
                w.wait()
            n = self.summary.export_marks(self.bufs[t], self.cap)
            self.cnt[t].fill_(n)
            if self.stage:
                if n:
                    self.hbufs[t][: 2 * n].copy_(self.bufs[t][: 2 * n])
                ops = [dist.P2POp(dist.isend, self.cnt[t], self._grank(0), group=self.group)]
                if n:
                    ops.append(dist.P2POp(dist.isend, self.hbufs[t][: 2 * n], self._grank(0), group=self.group))
            else:
                ops = [dist.P2POp(dist.isend, self.cnt[t], self._grank(0), group=self.group)]
                if n:
                    ops.append(dist.P2POp(dist.isend, self.bufs[t][: 2 * n], self._grank(0), group=self.group))
            self.works[t] = dist.batch_isend_irecv(ops)
            if self.stage:                             # gloo: the staging buffer is reused next turn
                for w in self.works[t]:
                    w.wait()
                self.works[t] = []
            self.turn ^= 1
            self.bytes_sent += 8 * n
            self.summary.close_window()
            return False
        # rank 0
        self.before_fold()
        for w in self._cnt_works:
            w.wait()
        self._cnt_works = None
        counts = [int(x) for x in self.cnts.tolist()]
        total = sum(counts)
        if max(counts) > self.cap:
            raise RuntimeError("a partial summary of %d pairs exceeds capacity %d" % (max(counts), self.cap))
        if total:
            if self.buf.numel() < 2 * total:
                if self.free_ev is not None:
                    self.free_ev.synchronize()
                self.buf = torch.empty(2 * total, dtype=torch.int32, device=self.device)
            dst = self.buf
            if self.stage:
                if self.hbuf.numel() < 2 * total:
                    self.hbuf = torch.empty(2 * total, dtype=torch.int32).pin_memory()
                dst = self.hbuf
            ops, off = [], 0
            for i, c in enumerate(counts):
                if c:
                    ops.append(dist.P2POp(dist.irecv, dst[2 * off: 2 * (off + c)], self._grank(i + 1), group=self.group))
                    off += c
            if self.side is not None:                  # transfers overlap this rank's fold
                if self.free_ev is not None:           # ... but not the previous fold out of self.buf
                    self.side.wait_event(self.free_ev)
                with torch.cuda.stream(self.side):
                    works = dist.batch_isend_irecv(ops)
            else:
                works = dist.batch_isend_irecv(ops)
            for w in works:
                w.wait()                               # NCCL: the current stream waits, not the host
            if self.stage:
                self.buf[: 2 * total].copy_(self.hbuf[: 2 * total])
            self.summary.fold_pairs(self.buf, total, id_bits=32)
            if self.side is not None:
                self.free_ev = torch.cuda.Event()
                self.free_ev.record(torch.cuda.current_stream(self.device))
            self.bytes_recv += 8 * total
        self.summary.close_window()
        return True

    def drain(self) -> None:
        """Wait for every send still in flight (before tearing the process group down)."""
        if self.rank != 0:
            for t in range(2):
                for w in self.works[t]:
                    w.wait()
                self.works[t] = []


# A receiver folding several ranks' deltas at once: while their big components are still separate
# (young windows) each delta must go in its own fold call, so that call's short head launch joins
# its components before the bulk arrives (csrc/cc_api.hip, merge_head); small deltas go in one call.
BULK_DELTA_PAIRS = 1 << 21


def fold_deltas(summary, buf, counts) -> None:
    """Fold the deltas laid out back to back in ``buf`` (counts[i] pairs each)."""
    total = sum(counts)
    if total == 0:
        return
    if max(counts) <= BULK_DELTA_PAIRS:
        summary.fold_pairs(buf, total, id_bits=32)
        return
    off = 0
    for c in counts:
        if c:
            summary.fold_pairs(buf[2 * off: 2 * (off + c)], c, id_bits=32)
            off += c


class AllgatherMerge:
    """Replicated global summary on every rank; per window an all-gather of deltas.

    Per window, every rank: export its marks (its slice's new connectivity relative to the global
    summary it held) into ``sendbuf``; all-gather the counts (one small collective, one host
    sync); pad its delta to the largest count m with copies of its first pair (a repeated union
    is a no-op) and all-gather the padded deltas (one collective: P slots of m pairs each, over
    every pair of GPUs' own xGMI link at once); fold the other ranks' slots with marking paused
    (they are the others' to export, not this rank's); close the window. All ranks then hold the
    same partition (the union of all ranks' edges); rank 0 reports the emission.
    One collective call instead of a batch of 2(P-1) send/recv ops keeps the host's share of the
    per-window critical path (the GPU idles from the count sync until the payload is enqueued)
    to one launch.
    Correctness argument: a delta holds (v, root(v)) for every root the exporting rank hooked and
    every self-loop first touch, so it carries every component join of that rank's window; joins
    are idempotent, so it applies to any summary of the same prior partition
    (tests/test_tree_gloo.py).
    The summary needs ``export_marks``, ``fold_pairs``, ``set_marking``, ``close_window`` and
    must have been created with marks tracked (GS_CC_TRACK_MARKS) on EVERY rank.
    """

    def __init__(self, summary, capacity_pairs: int, device: torch.device, group=None):
        self.summary = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.cap = int(capacity_pairs)
        self.stage = (dist.get_backend(group) == "gloo" and self.device.type == "cuda")
        cdev = "cpu" if (self.stage or self.device.type == "cpu") else self.device
        self.cnt = torch.zeros(1, dtype=torch.int64, device=cdev)
        self.cnts = torch.zeros(self.world, dtype=torch.int64, device=cdev)
        # device summaries export asynchronously into a device count (the collective's input
        # under RCCL; copied to the host first under gloo)
        self.dcnt = None
        if self.device.type == "cuda" and hasattr(summary, "export_marks_async"):
            self.dcnt = self.cnt if self.cnt.is_cuda else torch.zeros(1, dtype=torch.int64, device=self.device)
        # an export holds at most 2 x capacity pairs (include/gsgpu.h gs_cc_export_marks_async)
        self.sendbuf = torch.empty(4 * self.cap, dtype=torch.int32, device=self.device)
        self.recvbuf = torch.empty(2 * self.world, dtype=torch.int32, device=self.device)   # grows
        self.hsend = torch.empty(0, dtype=torch.int32)
        self.hrecv = torch.empty(0, dtype=torch.int32)
        self.bytes_sent = 0
        self.bytes_recv = 0
        # communicator up (all ranks take part) before the first window
        dist.all_gather_into_tensor(self.cnts, self.cnt, group=self.group)

    def _host(self, attr: str, n: int) -> torch.Tensor:
        t = getattr(self, attr)
        if t.numel() < n:
            t = torch.empty(max(n, 2 * t.numel()), dtype=torch.int32)
            if self.device.type == "cuda":
                t = t.pin_memory()
            setattr(self, attr, t)
        return t

    def _counts(self) -> List[int]:
        if self.dcnt is not None:
            # count straight from the device into the collective: one host sync per window
            self.summary.export_marks_async(self.sendbuf, self.dcnt)
            if self.stage:
                self.cnt.copy_(self.dcnt)
        else:
            self.cnt.fill_(self.summary.export_marks(self.sendbuf, self.cap))
        dist.all_gather_into_tensor(self.cnts, self.cnt, group=self.group)
        return [int(x) for x in self.cnts.tolist()]

    def merge_window(self) -> bool:
        if self.world == 1:
            self.summary.close_window()
            return True
        counts = self._counts()
        n, m, P = counts[self.rank], max(counts), self.world
        if m:
            if 0 < n < m:                                  # pad with copies of the first pair
                self.sendbuf[2 * n: 2 * m].view(-1, 2).copy_(self.sendbuf[0:2].view(1, 2).expand(m - n, 2))
            if self.recvbuf.numel() < 2 * P * m:
                self.recvbuf = torch.empty(2 * P * m, dtype=torch.int32, device=self.device)
            send, recv = self.sendbuf[: 2 * m], self.recvbuf[: 2 * P * m]
            if self.stage:                                 # gloo moves host tensors only
                hs = self._host("hsend", 2 * m)[: 2 * m]
                hs.copy_(send)
                hr = self._host("hrecv", 2 * P * m)[: 2 * P * m]
                dist.all_gather_into_tensor(hr, hs, group=self.group)
                recv.copy_(hr)
            else:
                dist.all_gather_into_tensor(recv, send, group=self.group)
            self.bytes_sent += 8 * m * (P - 1)
            self.bytes_recv += 8 * m * (P - 1)
            self.summary.set_marking(False)
            fold_slots(self.summary, recv, m, [0 if q == self.rank else c for q, c in enumerate(counts)])
            self.summary.set_marking(True)
        self.summary.close_window()
        return self.rank == 0


def fold_slots(summary, buf, m: int, counts) -> None:
    """Fold deltas laid out in slots of m pairs (slot q: counts[q] real pairs, then copies of its
    first pair). Only the real pairs are folded, as the C-ABI exchange's slot fold reads each slot's
    count (k_fold_slots): the copies are no-op unions, but folding them put up to (m - counts[q])
    lanes on one claim CAS — a same-address herd the real protocol does not have (the rank model's
    all-gather window 5: 2.3 ms for 1.4 M pairs). While the deltas are big (young windows,
    components not yet joined) each slot goes in its own call, so that call's short head launch
    joins its components before the bulk (see fold_deltas); otherwise the slots' real pairs are
    packed into one call."""
    if max(counts) > BULK_DELTA_PAIRS:
        for q, c in enumerate(counts):
            if c:
                summary.fold_pairs(buf[2 * q * m: 2 * (q * m + c)], c, id_bits=32)
        return
    parts = [buf[2 * q * m: 2 * (q * m + c)] for q, c in enumerate(counts) if c]
    if not parts:
        return
    packed = parts[0] if len(parts) == 1 else torch.cat(parts)
    summary.fold_pairs(packed, packed.numel() // 2, id_bits=32)


class PrefilterMerge:
    """GS_MERGE_PREFILTER restated over torch.distributed (csrc/comm.hip merge_prefilter): rank 0
    is the Merger (the summary); ranks 1..P-1 keep only a giant bitmap — the component rank 0
    broadcasts after its closes of windows w < BCAST_YOUNG and every BCAST_EVERY-th — and send the
    edges of their slice that are NOT inside it (count, then the pairs) to rank 0, which folds its
    own slice and everyone's survivors and closes. The giant here is the largest component at the
    close (the device samples it; any component is correct: a stale or switched bitmap only lets
    more edges through, components only merge). ``merge_window(src, dst)`` takes this rank's slice
    of the window (rank 0 has folded its own already) and returns True on rank 0."""
    BCAST_YOUNG, BCAST_EVERY = 4, 16

    def __init__(self, summary, capacity: int, device: torch.device, group=None):
        self.summary, self.cap, self.device, self.group = summary, int(capacity), device, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.gbits = torch.zeros(self.cap, dtype=torch.uint8, device=device)
        self.win = 0
        self.survivors_sent = 0

    def _g(self, r: int) -> int:
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _pick(self) -> None:
        p = self.summary.parent
        seen = p >= 0
        if not seen.any():
            self.gbits.zero_()
            return
        self.summary.close_window()
        roots = p[seen]
        vals, cnt = np.unique(roots, return_counts=True)
        g = vals[int(np.argmax(cnt))]
        self.gbits.copy_(torch.from_numpy((p == g).astype(np.uint8)))

    def merge_window(self, src, dst) -> bool:
        w, self.win = self.win, self.win + 1
        if self.rank != 0:
            s = np.asarray(src, dtype=np.int64)
            d = np.asarray(dst, dtype=np.int64)
            gb = self.gbits.cpu().numpy().astype(bool)
            keep = ~(gb[s] & gb[d])
            pairs = np.empty(2 * int(keep.sum()), dtype=np.int64)
            pairs[0::2], pairs[1::2] = s[keep], d[keep]
            n = torch.tensor([pairs.size // 2], dtype=torch.int64, device=self.device)
            dist.send(n, self._g(0), group=self.group)
            if pairs.size:
                dist.send(torch.from_numpy(pairs).to(self.device), self._g(0), group=self.group)
            self.survivors_sent += pairs.size // 2
        else:
            for q in range(1, self.world):
                n = torch.zeros(1, dtype=torch.int64, device=self.device)
                dist.recv(n, self._g(q), group=self.group)
                if int(n.item()):
                    buf = torch.empty(2 * int(n.item()), dtype=torch.int64, device=self.device)
                    dist.recv(buf, self._g(q), group=self.group)
                    b = buf.cpu().numpy()
                    self.summary.fold(b[0::2], b[1::2])
            self.summary.close_window()
        if w < self.BCAST_YOUNG or w % self.BCAST_EVERY == self.BCAST_EVERY - 1:
            if self.rank == 0:
                self._pick()
            dist.broadcast(self.gbits, self._g(0), group=self.group)
        return self.rank == 0
