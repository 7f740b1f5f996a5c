"""BipartitenessCheck on the device (include/gsgpu.h gs_bip_*): Python mirror of the reference's
``library/BipartitenessCheck.java:38-133`` operator and its ``summaries/Candidates.java`` summary.

``Candidates`` holds one device summary (union-find with a parity bit per vertex);
``BipartitenessCheck(mergeWindowTime)`` runs the SummaryBulkAggregation dataflow over a
``SimpleEdgeStream`` and yields the cumulative summary after every window, whose ``toString()``
is the reference's emission format, e.g. ``(true,{1={1=(1,true), 2=(2,false)}})`` or
``(false,{})`` (BipartitenessCheckTest.java:45-48, :70-72).

``Candidates(..., literal=True)`` / ``BipartitenessCheck(..., mode="literal")``: the reference's
Candidates.merge rule as written (GS_BIP_REFERENCE_LITERAL, csrc/bip_literal.hpp), whose emissions
differ from the intended semantics on multi-window and multi-partition streams (a vertex can sit
in several components, keys can be signed false); the dataflow is then the reference's own (fresh
partial per partition per window, combined in partition order, the Merger's
``windowResult.merge(summary)``), since the literal rule depends on it.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

from . import _abi
from ._abi import call
from .summary import _buf, _stream_ptr

U64 = ctypes.c_uint64


class Candidates:
    """Candidates (summaries/Candidates.java:25-197) on the device; ids in [0, capacity)."""

    def __init__(self, vertex_capacity: int, id_bits: int = 64, device: int = 0, stream=None,
                 literal: bool = False, entry_capacity: int = 0):
        self.capacity = int(vertex_capacity)
        self.id_bits = int(id_bits)
        self.literal = bool(literal)
        h = ctypes.c_void_p()
        call("gs_bip_create_ex", ctypes.byref(h), self.capacity, self.id_bits, int(device),
             _abi.GS_BIP_REFERENCE_LITERAL if literal else 0, int(entry_capacity))
        self._h = h
        if stream is not None:
            call("gs_bip_set_stream", self._h, _stream_ptr(stream))

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise RuntimeError("Candidates is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            _abi.lib().gs_bip_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass

    def reset(self) -> None:
        """Back to ``new Candidates(true)``."""
        call("gs_bip_reset", self.handle)

    def fold(self, src, dst) -> None:
        """updateFunction.foldEdges over a batch: merge(edgeToCandidate(u, v)) per edge."""
        ps, ks, n = _buf(src, self.id_bits, "src")
        pd, kd, m = _buf(dst, self.id_bits, "dst")
        if n != m:
            raise ValueError("src and dst lengths differ (%d, %d)" % (n, m))
        call("gs_bip_fold", self.handle, ps, pd, n)

    def merge(self, other: "Candidates") -> "Candidates":
        """Candidates.merge(input) (:70-128): returns this summary, which absorbed ``other``."""
        call("gs_bip_merge", self.handle, other.handle)
        return self

    def close_window(self) -> None:
        call("gs_bip_close_window", self.handle)

    def sync(self) -> None:
        call("gs_bip_sync", self.handle)

    def status(self) -> Tuple[bool, int, int]:
        ok, nv, nc = ctypes.c_int(), U64(), U64()
        call("gs_bip_status", self.handle, ctypes.byref(ok), ctypes.byref(nv), ctypes.byref(nc))
        return bool(ok.value), int(nv.value), int(nc.value)

    def getSuccess(self) -> bool:
        """Candidates.getSuccess (:40-42)."""
        return self.status()[0]

    def checksum(self) -> Tuple[int, bool, int, int]:
        s, ok, nv, nc = U64(), ctypes.c_int(), U64(), U64()
        call("gs_bip_checksum", self.handle, ctypes.byref(s), ctypes.byref(ok), ctypes.byref(nv), ctypes.byref(nc))
        return int(s.value), bool(ok.value), int(nv.value), int(nc.value)

    def pairs(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(vertices, keys, signs) of every vertex, ordered by vertex (literal summaries: every
        (component, vertex) entry, ordered by vertex then key)."""
        nv = self.status()[1]
        dt = np.uint32 if self.id_bits == 32 else np.int64
        v = np.empty(max(nv, 1), dtype=dt)
        k = np.empty(max(nv, 1), dtype=dt)
        sg = np.empty(max(nv, 1), dtype=np.uint8)
        got = U64()
        call("gs_bip_emit_pairs", self.handle, v.ctypes.data_as(ctypes.c_void_p), k.ctypes.data_as(ctypes.c_void_p),
             sg.ctypes.data_as(ctypes.c_void_p), nv, ctypes.byref(got))
        n = int(got.value)
        return v[:n].astype(np.int64), k[:n].astype(np.int64), sg[:n].astype(bool)

    def getMap(self) -> Dict[int, Dict[int, bool]]:
        """Candidates.getMap (:44-46): component key -> {vertex: sign}; empty once failed."""
        ok, _, _ = self.status()
        if not ok:
            return {}
        out: Dict[int, Dict[int, bool]] = {}
        v, k, s = self.pairs()
        for a, b, c in zip(v.tolist(), k.tolist(), s.tolist()):
            out.setdefault(b, {})[a] = c
        return out

    # ---- checkpoint / resume (the Merger's ListCheckpointed state, SummaryAggregation.java:127-135) ----
    def snapshot(self) -> Tuple[bool, np.ndarray, np.ndarray, np.ndarray]:
        """(success, vertices, keys, signs): everything a Candidates serialises (Candidates.java:27)."""
        ok = self.getSuccess()
        if not ok:
            e = np.empty(0, dtype=np.int64)
            return False, e, e, np.empty(0, dtype=bool)
        v, k, s = self.pairs()
        return True, v, k, s

    def restore(self, success, vertices, keys, signs) -> None:
        """This summary becomes the snapshotted one (gs_bip_restore). A reference-literal summary
        loads the entries as they are (its components may share vertices); an intended one is
        rebuilt from one parity edge per vertex, relative to its component key's own sign
        (reversed merges can leave a key signed false, Candidates.java:155-182): a vertex signed
        differently from its key gets the edge (v, key); a vertex signed like its key (other than
        the key) gets an edge to a vertex of its component signed the other way (a connected
        bipartite component of several vertices has one); a lone key gets its self-loop
        (edgeToCandidate(v, v) adds it). A failed snapshot is restored as failed
        (Candidates.fail(): empty map; intended summaries: an odd cycle on ids 0..2)."""
        dt = np.uint32 if self.id_bits == 32 else np.int64
        v = np.asarray(vertices, dtype=np.int64)
        k = np.asarray(keys, dtype=np.int64)
        s = np.asarray(signs, dtype=bool)
        if not (v.shape == k.shape == s.shape):
            raise ValueError("restore: vertices, keys and signs differ in length")
        if not success:
            v = k = np.empty(0, dtype=np.int64)
            s = np.empty(0, dtype=bool)
        if v.size and (v.min() < 0 or k.min() < 0):
            raise ValueError("restore: negative vertex id")
        va = np.ascontiguousarray(v.astype(dt))
        ka = np.ascontiguousarray(k.astype(dt))
        sa = np.ascontiguousarray(s.astype(np.uint8))
        call("gs_bip_restore", self.handle, 1 if success else 0, va.ctypes.data_as(ctypes.c_void_p),
             ka.ctypes.data_as(ctypes.c_void_p), sa.ctypes.data_as(ctypes.c_void_p), int(va.size))

    def toString(self) -> str:
        """Tuple2<Boolean, TreeMap<Long, TreeMap<Long, SignedVertex>>>.toString."""
        ok = self.getSuccess()
        if not ok:
            return "(false,{})"
        m = self.getMap()
        return "(true,{%s})" % ", ".join(
            "%d={%s}" % (key, ", ".join("%d=(%d,%s)" % (v, v, "true" if s else "false") for v, s in sorted(c.items())))
            for key, c in sorted(m.items()))

    __str__ = toString


class BipartitenessCheck:
    """BipartitenessCheck(mergeWindowTime) (BipartitenessCheck.java:50-52): the
    SummaryBulkAggregation dataflow with initial value Candidates(true), transientState false.

    mode "fused" folds every window into the one cumulative summary (production: the check and
    its bipartition do not depend on the partitioning); mode "reference" folds P fresh partials
    per window, combines them with Candidates.merge in partition order and lets the Merger merge
    the window result with the cumulative summary (SummaryAggregation.java:106-119); mode
    "literal" runs that same dataflow on reference-literal summaries (Candidates.java:77-192 as
    written: the reference's own emissions, multi-window quirks included)."""

    def __init__(self, mergeWindowTime: int, *, vertex_capacity: Optional[int] = None, id_bits: int = 64,
                 device: int = 0, parallelism: int = 1, window_edges: Optional[int] = None, mode: str = "fused",
                 entry_capacity: int = 0):
        if mode not in ("fused", "reference", "literal"):
            raise ValueError("mode must be 'fused', 'reference' or 'literal'")
        self.entry_capacity = int(entry_capacity)
        self.time_millis = int(mergeWindowTime)
        self.vertex_capacity = vertex_capacity
        self.id_bits = int(id_bits)
        self.device = int(device)
        self.parallelism = max(int(parallelism), 1)
        self.window_edges = window_edges
        self.mode = mode
        self._summary: Optional[Candidates] = None     # the Merger's cumulative summary
        self._restored = None                          # restoreState's snapshot, for the next run

    # ---- Merger checkpointing (ListCheckpointed<S>, SummaryAggregation.java:127-135) ----
    def snapshotState(self, checkpointId: int = 0, timestamp: int = 0) -> list:
        """Collections.singletonList(summary); empty before the first emission."""
        if self._summary is None:
            return []
        return [self._summary.snapshot()]

    def restoreState(self, state: list) -> None:
        """summary = list.get(0): the next run() starts its Merger from this snapshot."""
        self._restored = state[0] if state else None

    def _capacity(self, stream) -> int:
        if self.vertex_capacity:
            return int(self.vertex_capacity)
        hi = 0 if len(stream) == 0 else int(max(stream.src.max(), stream.dst.max())) + 1
        if self._restored is not None and len(self._restored[1]):
            hi = max(hi, int(np.max(self._restored[1])) + 1)
        if self._restored is not None and not self._restored[0]:
            hi = max(hi, 3)                            # a failed snapshot is restored on ids 0..2
        return max(hi, 1)

    def run(self, stream) -> Iterator[Candidates]:
        cap = self._capacity(stream)
        wins = stream.windows(self.time_millis, self.window_edges)
        if self.mode == "fused":
            summary = Candidates(cap, self.id_bits, self.device)
            if self._restored is not None:
                summary.restore(*self._restored)
            self._summary = summary
            try:
                for w in wins:
                    summary.fold(stream.src[w], stream.dst[w])
                    summary.close_window()
                    yield summary
            finally:
                self._summary = None
                summary.close()
            return
        P = self.parallelism
        lit = self.mode == "literal"
        pool: List[Candidates] = [Candidates(cap, self.id_bits, self.device, literal=lit,
                                             entry_capacity=self.entry_capacity) for _ in range(P + 1)]
        summary: Optional[Candidates] = None
        if self._restored is not None:                 # restoreState: the Merger resumes from it
            summary = pool[P]
            summary.restore(*self._restored)
        try:
            for w in wins:
                lo, ln = w.start, w.stop - w.start
                free = [c for c in pool if c is not summary]
                acc: Optional[Candidates] = None
                for p in range(P):
                    a, b = lo + (ln * p) // P, lo + (ln * (p + 1)) // P
                    if a == b:
                        continue
                    part = free.pop()
                    part.reset()
                    part.fold(stream.src[a:b], stream.dst[a:b])
                    acc = part if acc is None else acc.merge(part)       # combineFunction.reduce(c1, c2) = c1.merge(c2)
                summary = acc if summary is None else acc.merge(summary)  # Merger: reduce(windowResult, summary)
                summary.close_window()
                self._summary = summary
                yield summary
        finally:
            self._summary = None
            for c in pool:
                c.close()
