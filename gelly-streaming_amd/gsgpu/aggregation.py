"""Host-side mirror of the reference's streaming operator surface for Connected Components.

Reference (paths relative to src/main/java/org/apache/flink/graph/streaming/):

* ``SimpleEdgeStream.aggregate(summaryAggregation)`` -> ``summaryAggregation.run(edges)``
  (SimpleEdgeStream.java:100-102, GraphStream.java:139-140)
* ``SummaryBulkAggregation(updateFun, combineFun, initialVal, timeMillis, transientState)``
  (SummaryBulkAggregation.java:57-64) and its dataflow ``run`` (:68-90): per-partition
  tumbling-window fold from a fresh initial value, ``timeWindowAll`` reduce with the combine
  function, then the parallelism-1 ``Merger`` (SummaryAggregation.java:106-119) that folds each
  window result into the cumulative summary and emits it.
* ``ConnectedComponents(long mergeWindowTime)`` (library/ConnectedComponents.java:52-54).

Windows: the reference's are wall-clock / event-time tumbling windows. Here a stream carries
either event timestamps (window = floor(ts / mergeWindowTime), Flink's tumbling window
assignment with offset 0) or none, in which case ``window_edges`` cuts count-based windows
(SURVEY.md §7 "Hard parts"). Partition p of a window is its contiguous slice
[p*len/P, (p+1)*len/P), as in oracle/pipeline.c.

Modes:
* ``mode="fused"`` (default, the production path on one GPU): every window's edges, whatever
  partition they belong to, are folded straight into the one cumulative device summary and the
  window is closed (compressed) before its emission. The emitted canonical labels equal the
  reference's, which do not depend on partitioning, merge order or rank tie-breaks (union-find
  over the union of all edges so far).
* ``mode="reference"``: the reference dataflow step by step on the device — one fresh partial
  summary per partition per window, ``CombineCC`` in partition order, then the Merger's
  ``CombineCC(windowResult, summary)``. Used by the parity tests of ``CombineCC``.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Sequence

import numpy as np

from .summary import CombineCC, DisjointSet, UpdateCC


class SimpleEdgeStream:
    """An edge stream in arrival order: src[i] -> dst[i], optional event timestamps (ms)."""

    def __init__(self, src, dst, timestamps: Optional[Sequence[int]] = None):
        self.src = np.ascontiguousarray(np.asarray(src, dtype=np.int64))
        self.dst = np.ascontiguousarray(np.asarray(dst, dtype=np.int64))
        if self.src.shape != self.dst.shape:
            raise ValueError("src/dst length mismatch")
        self.timestamps = None if timestamps is None else np.asarray(timestamps, dtype=np.int64)
        if self.timestamps is not None and self.timestamps.shape != self.src.shape:
            raise ValueError("timestamps length mismatch")

    def __len__(self) -> int:
        return int(self.src.size)

    def aggregate(self, summary_aggregation: "SummaryBulkAggregation") -> Iterator[DisjointSet]:
        """GraphStream.aggregate (GraphStream.java:139-140)."""
        return summary_aggregation.run(self)

    def windows(self, time_millis: int, window_edges: Optional[int]) -> List[slice]:
        n = len(self)
        if n == 0:
            return []
        if self.timestamps is not None and not window_edges:
            if np.any(np.diff(self.timestamps) < 0):
                raise ValueError("timestamps must be ascending (AscendingTimestampExtractor)")
            wid = self.timestamps // int(time_millis)
            cuts = np.nonzero(np.diff(wid))[0] + 1
            bounds = [0] + cuts.tolist() + [n]
            return [slice(a, b) for a, b in zip(bounds[:-1], bounds[1:])]
        w = int(window_edges) if window_edges else n
        return [slice(a, min(a + w, n)) for a in range(0, n, w)]


class SummaryBulkAggregation:
    """Partitioned fold -> windowAll combine -> Merger (SummaryBulkAggregation.java:68-90)."""

    def __init__(self, update_fun: UpdateCC, combine_fun: CombineCC, time_millis: int,
                 transient_state: bool, *, vertex_capacity: Optional[int] = None, id_bits: int = 64,
                 device: int = 0, parallelism: int = 1, window_edges: Optional[int] = None,
                 mode: str = "fused", sparse: Optional[bool] = None):
        if mode not in ("fused", "reference"):
            raise ValueError("mode must be 'fused' or 'reference'")
        self.update_fun = update_fun
        self.combine_fun = combine_fun
        self.time_millis = int(time_millis)
        self.transient_state = bool(transient_state)
        self.vertex_capacity = vertex_capacity
        self.id_bits = id_bits
        self.device = device
        self.parallelism = max(int(parallelism), 1)
        self.window_edges = window_edges
        self.mode = mode
        self.sparse = sparse          # None: sparse ids (GS_CC_SPARSE_IDS) iff some id is < 0 or >= 2^32 - 1
        self._summary: Optional[DisjointSet] = None      # the Merger's cumulative summary
        self._restored = None                            # restoreState's snapshot, for the next run

    # ---- Merger checkpointing (ListCheckpointed<S>, SummaryAggregation.java:127-135) ----
    def snapshotState(self, checkpointId: int = 0, timestamp: int = 0) -> list:
        """Collections.singletonList(summary): the cumulative summary as canonical
        (vertices, labels); an empty list before the first emission (summary == initialVal)."""
        if self._summary is None:
            return []
        return [self._summary.snapshot()]

    def restoreState(self, state: list) -> None:
        """summary = list.get(0): the next run() starts its Merger from this snapshot."""
        self._restored = state[0] if state else None

    def _use_sparse(self, stream: SimpleEdgeStream) -> bool:
        if self.sparse is not None:
            return bool(self.sparse)
        if self.id_bits != 64 or len(stream) == 0:
            return False
        lo = min(int(stream.src.min()), int(stream.dst.min()))
        hi = max(int(stream.src.max()), int(stream.dst.max()))
        if self._restored is not None and len(self._restored[0]):
            rv = np.asarray(self._restored[0], dtype=np.int64)
            lo, hi = min(lo, int(rv.min())), max(hi, int(rv.max()))
        return lo < 0 or hi >= 0xFFFFFFFF

    def _capacity(self, stream: SimpleEdgeStream) -> int:
        if self.vertex_capacity:
            return int(self.vertex_capacity)
        if len(stream) == 0:
            return 1
        if self._sparse_run:
            return int(np.unique(np.concatenate([stream.src, stream.dst])).size)
        return int(max(stream.src.max(), stream.dst.max())) + 1

    def _new(self, cap: int) -> DisjointSet:
        return DisjointSet(cap, id_bits=self.id_bits, device=self.device, sparse=self._sparse_run)

    def run(self, stream: SimpleEdgeStream) -> Iterator[DisjointSet]:
        self._sparse_run = self._use_sparse(stream)
        cap = self._capacity(stream)
        if self._restored is not None and len(self._restored[0]) and not self.vertex_capacity:
            rv = np.asarray(self._restored[0], dtype=np.int64)
            if self._sparse_run:                  # distinct ids of the stream and the snapshot
                ids = [rv] + ([stream.src, stream.dst] if len(stream) else [])
                cap = int(np.unique(np.concatenate(ids)).size)
            else:
                cap = max(cap, int(rv.max()) + 1)
        wins = stream.windows(self.time_millis, self.window_edges)
        if self.mode == "fused":
            yield from self._run_fused(stream, wins, cap)
        else:
            yield from self._run_reference(stream, wins, cap)

    def _run_fused(self, stream, wins, cap) -> Iterator[DisjointSet]:
        summary = self._new(cap)
        if self._restored is not None:
            summary.restore(*self._restored)
        self._summary = summary
        try:
            for w in wins:
                if self.transient_state:
                    summary.reset()
                self.update_fun.fold_batch(summary, stream.src[w], stream.dst[w])
                summary.close_window()
                yield summary                      # Merger: collector.collect(summary)
        finally:
            self._summary = None
            summary.close()

    def _run_reference(self, stream, wins, cap) -> Iterator[DisjointSet]:
        P = self.parallelism
        pool = [self._new(cap) for _ in range(P + 1)]
        summary: Optional[DisjointSet] = None     # Merger.summary = initialVal (empty)
        if self._restored is not None:            # restoreState: the Merger resumes from it
            summary = pool[P]
            summary.restore(*self._restored)
        try:
            for w in wins:
                lo, ln = w.start, w.stop - w.start
                free = [d for d in pool if d is not summary]
                acc: Optional[DisjointSet] = None
                for p in range(P):
                    a, b = lo + (ln * p) // P, lo + (ln * (p + 1)) // P
                    if a == b:
                        continue                   # no element -> no window result
                    part = free.pop()
                    part.reset()                   # fresh copy of the initial value
                    self.update_fun.fold_batch(part, stream.src[a:b], stream.dst[a:b])
                    acc = part if acc is None else self.combine_fun.reduce(acc, part)
                if summary is None or self.transient_state:
                    summary = acc                  # reduce(s, empty) returns s
                else:
                    summary = self.combine_fun.reduce(acc, summary)
                summary.close_window()
                self._summary = summary
                yield summary
        finally:
            self._summary = None
            for d in pool:
                d.close()


class ConnectedComponents(SummaryBulkAggregation):
    """ConnectedComponents(long mergeWindowTime) (library/ConnectedComponents.java:52-54):
    UpdateCC, CombineCC, a new DisjointSet as initial value, transientState = false."""

    def __init__(self, mergeWindowTime: int, **kw):
        super().__init__(UpdateCC(), CombineCC(), mergeWindowTime, False, **kw)


class SummaryTreeReduce(SummaryBulkAggregation):
    """Partitioned fold -> log2 pairwise tree of combines -> windowAll combine -> Merger.

    SummaryTreeReduce.java:68-123: partial summaries of `degree` partitions are combined in
    rounds keyed by ``partition / 2`` (pairs (2i, 2i+1) meet at subtask i) while more than two
    remain (``enhance``, :95-123), then the last ones go through ``timeWindowAll`` reduce and the
    Merger (:87-90). Here every partial is a device summary and every combine is CombineCC
    (gs_cc_combine); the canonical emission equals the bulk aggregation's.
    """

    def __init__(self, update_fun: UpdateCC, combine_fun: CombineCC, time_millis: int,
                 transient_state: bool, degree: int = -1, **kw):
        kw.setdefault("mode", "reference")
        super().__init__(update_fun, combine_fun, time_millis, transient_state, **kw)
        if degree != -1:
            self.parallelism = max(int(degree), 1)
        self.degree = self.parallelism

    def _run_reference(self, stream, wins, cap) -> Iterator[DisjointSet]:
        P = self.parallelism
        pool = [self._new(cap) for _ in range(P + 1)]
        summary: Optional[DisjointSet] = None     # Merger.summary = initialVal (empty)
        if self._restored is not None:            # restoreState: the Merger resumes from it
            summary = pool[P]
            summary.restore(*self._restored)
        try:
            for w in wins:
                lo, ln = w.start, w.stop - w.start
                free = [d for d in pool if d is not summary]
                level: List[Optional[DisjointSet]] = []
                for p in range(P):
                    a, b = lo + (ln * p) // P, lo + (ln * (p + 1)) // P
                    if a == b:
                        level.append(None)                 # no element -> no window result
                        continue
                    part = free.pop()
                    part.reset()
                    self.update_fun.fold_batch(part, stream.src[a:b], stream.dst[a:b])
                    level.append(part)
                while len(level) > 2:                      # enhance(): key = partition / 2
                    nxt: List[Optional[DisjointSet]] = []
                    for i in range(0, len(level), 2):
                        x = level[i]
                        y = level[i + 1] if i + 1 < len(level) else None
                        if x is None or y is None:
                            nxt.append(x if y is None else y)
                        else:
                            nxt.append(self.combine_fun.reduce(x, y))
                    level = nxt
                acc: Optional[DisjointSet] = None          # windowAll reduce of what is left
                for x in level:
                    if x is not None:
                        acc = x if acc is None else self.combine_fun.reduce(acc, x)
                if summary is None or self.transient_state:
                    summary = acc
                else:
                    summary = self.combine_fun.reduce(acc, summary)
                summary.close_window()
                self._summary = summary            # what snapshotState serialises (ListCheckpointed)
                yield summary
        finally:
            self._summary = None
            for d in pool:
                d.close()


class ConnectedComponentsTree(SummaryTreeReduce):
    """ConnectedComponentsTree(long mergeWindowTime[, int degree])
    (library/ConnectedComponentsTree.java:28-34)."""

    def __init__(self, mergeWindowTime: int, degree: int = -1, **kw):
        super().__init__(UpdateCC(), CombineCC(), mergeWindowTime, False, degree, **kw)
