"""TEST INFRASTRUCTURE ONLY — CPU oracle of the reference's BipartitenessCheck (parity checker).

Only tests/ may import this module; the product path (libgsgpu.so, gs_bip_*) never does.

Two restatements live here:

* ``LiteralCandidates`` + ``literal_run`` — line by line the reference's summary and dataflow:
  summaries/Candidates.java:25-197 (success flag + TreeMap component key -> TreeMap vertex ->
  SignedVertex), library/BipartitenessCheck.java:50-133 (edgeToCandidate :54-61, foldEdges
  :93-95, combineFunction :121-124), SummaryBulkAggregation.java:68-130 (fresh Candidates(true)
  per partition per window, windowAll reduce) and SummaryAggregation.java:106-119 (Merger:
  summary = combine(windowResult, summary), transientState = false). Pure Python: small cases.
* ``ParityUnionFind`` / ``intended_run`` — the semantics the reference's own tests pin
  (T/example/test/BipartitenessCheckTest.java:35-90): the stream so far is bipartite or not;
  when it is, every component keyed by its minimum vertex id, every vertex signed true iff it
  is on the key vertex's side; a self-loop only adds its vertex (edgeToCandidate(v, v): the
  second add is refused and the refusal ignored). Union-find with parity; cross-checked
  against a BFS 2-colouring (``bfs_bipartition``).

Where they differ. Candidates.merge (Candidates.java:71-128) folds an input component into the
LOWEST-keyed overlapping candidate component `firstKey`, but writes the merged vertices under
min(inputKey, firstKey) (:167-181) and removes only mergeWith[1..] (:117-126): when the input
key is smaller than firstKey, the old firstKey component stays beside the new one and shares
vertices with it; a failed merge of those (:121-123) calls fail() without returning it (an odd
cycle can then go unreported); and the merged component keeps the SELF side's signs, so the key
vertex can be signed false. The Merger merges the cumulative summary into each new window's
candidates (SummaryAggregation.java:110: reduce(windowResult, summary) = window.merge(summary)),
so from the second window on the older, smaller-keyed component is the input and all three
effects appear. With one window and one partition and a stream in which no edge's smaller
endpoint undercuts the key of the component it joins — the setting of the reference's own
tests — the literal restatement equals the intended semantics (tests/test_bipartite_oracle.py);
the GPU path implements the intended semantics, pinned by the reference's two known answers,
and the literal restatement documents where the reference departs from them.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np


# ------------------------------------------------------------------------------------------
# literal restatement of Candidates.java / BipartitenessCheck.java
# ------------------------------------------------------------------------------------------
class LiteralCandidates:
    """Tuple2<Boolean, TreeMap<Long, Map<Long, SignedVertex>>>; SignedVertex = (vertex, sign)."""

    def __init__(self, success: bool = True):          # Candidates(boolean) :30-33
        self.f0 = success
        self.f1: Dict[int, Dict[int, bool]] = {}

    def add_component(self, component: int, vertices: Dict[int, bool]) -> bool:   # :46-53
        for v, sign in list(vertices.items()):
            if not self.add(component, v, sign):
                return False
        return True

    def add(self, component: int, vertex: int, sign: bool) -> bool:                # :55-67
        comp = self.f1.setdefault(component, {})
        if vertex in comp and comp[vertex] != sign:
            return False
        comp[vertex] = sign
        return True

    def merge(self, inp: "LiteralCandidates") -> "LiteralCandidates":            # :70-128
        if not inp.f0 or not self.f0:
            return LiteralCandidates(False)
        for in_key in sorted(inp.f1):
            in_comp = inp.f1[in_key]
            merge_with: List[int] = []
            for self_key in sorted(self.f1):
                self_comp = self.f1[self_key]
                if set(in_comp) == set(self_comp):                               # :84-87
                    continue
                for v in sorted(in_comp):                                        # :90-97
                    if v in self_comp:
                        if self_key not in merge_with:
                            merge_with.append(self_key)
                            break
            if not merge_with:
                self.add_component(in_key, in_comp)                              # :103
            else:
                merge_with.sort()
                first = merge_with[0]
                if not LiteralCandidates._merge(inp, self, in_key, first):
                    return LiteralCandidates(False)
                first = min(in_key, first)
                for k in merge_with[1:]:
                    LiteralCandidates._merge(self, self, k, first)               # result dropped (:121-123)
                    self.f1.pop(k, None)
        return self

    @staticmethod
    def _merge(inp: "LiteralCandidates", cands: "LiteralCandidates", in_key: int, self_key: int) -> bool:  # :133-185
        in_comp = inp.f1[in_key]
        self_comp = cands.f1[self_key]
        merge_by = [v for v in sorted(in_comp) if v in self_comp]
        reversed_ = in_comp[merge_by[0]] != self_comp[merge_by[0]]
        for v in merge_by:
            ok = (in_comp[v] != self_comp[v]) if reversed_ else (in_comp[v] == self_comp[v])
            if not ok:
                return False
        common = min(in_key, self_key)
        for v in sorted(in_comp):
            sign = in_comp[v]
            if not cands.add(common, v, (not sign) if reversed_ else sign):
                return False
        return True

    def to_string(self) -> str:
        """Tuple2.toString of (Boolean, TreeMap<Long, TreeMap<Long, SignedVertex>>)."""
        comps = ", ".join("%d={%s}" % (k, ", ".join("%d=(%d,%s)" % (v, v, "true" if s else "false")
                                                     for v, s in sorted(self.f1[k].items())))
                          for k in sorted(self.f1))
        return "(%s,{%s})" % ("true" if self.f0 else "false", comps)


def edge_to_candidate(v1: int, v2: int) -> LiteralCandidates:                    # BipartitenessCheck.java:54-61
    src, trg = min(v1, v2), max(v1, v2)
    c = LiteralCandidates(True)
    c.add(src, src, True)
    c.add(src, trg, False)
    return c


def literal_run(src, dst, window_edges: int, partitions: int = 1) -> List[str]:
    """SummaryBulkAggregation + Merger over count windows; partition p folds the contiguous
    slice p of each window; returns the emission (toString) after every window."""
    n = len(src)
    W = window_edges if window_edges > 0 else max(n, 1)
    summary: Optional[LiteralCandidates] = None
    out = []
    for lo in range(0, n, W):
        hi = min(lo + W, n)
        parts = []
        for p in range(partitions):
            a = lo + (hi - lo) * p // partitions
            b = lo + (hi - lo) * (p + 1) // partitions
            if a == b:
                continue
            c = LiteralCandidates(True)
            for i in range(a, b):
                c = c.merge(edge_to_candidate(int(src[i]), int(dst[i])))         # foldEdges :93-95
            parts.append(c)
        window = parts[0]
        for c in parts[1:]:
            window = window.merge(c)                                              # combineFunction :121-124
        summary = window if summary is None else window.merge(summary)            # Merger: combine(windowResult, summary)
        out.append(summary.to_string())
    return out


# ------------------------------------------------------------------------------------------
# intended semantics (what the reference's tests pin): union-find with parity
# ------------------------------------------------------------------------------------------
class ParityUnionFind:
    def __init__(self):
        self.parent: Dict[int, int] = {}
        self.par: Dict[int, int] = {}          # parity of v relative to parent[v]
        self.ok = True

    def find(self, x: int) -> Tuple[int, int]:
        path = []
        while self.parent[x] != x:
            path.append(x)
            x = self.parent[x]
        root = x
        acc = 0
        for v in reversed(path):               # compress, accumulating parity to the root
            acc ^= self.par[v]
            self.par[v] = acc
            self.parent[v] = root
        return root, (self.par[path[0]] if path else 0)

    def union(self, u: int, v: int) -> None:
        for x in (u, v):
            if x not in self.parent:
                self.parent[x] = x
                self.par[x] = 0
        if not self.ok or u == v:           # self-loop: edgeToCandidate adds (v, true) only
            return
        ru, pu = self.find(u)
        rv, pv = self.find(v)
        if ru == rv:
            if pu == pv:
                self.ok = False
            return
        hi, lo = (ru, rv) if ru > rv else (rv, ru)
        self.parent[hi] = lo
        self.par[hi] = pu ^ pv ^ 1

    def emission(self) -> Tuple[bool, Dict[int, int], Dict[int, bool]]:
        """(bipartite, key[v] = min id of v's component, sign[v] = same side as the key)."""
        if not self.ok:
            return False, {}, {}
        key, sign = {}, {}
        for v in self.parent:
            r, p = self.find(v)
            key[v] = r                          # roots are component minima (smaller root wins)
            sign[v] = p == 0
        return True, key, sign


def emission_string(ok: bool, key: Dict[int, int], sign: Dict[int, bool]) -> str:
    if not ok:
        return "(false,{})"
    comps: Dict[int, List[int]] = {}
    for v, k in key.items():
        comps.setdefault(k, []).append(v)
    return "(true,{%s})" % ", ".join(
        "%d={%s}" % (k, ", ".join("%d=(%d,%s)" % (v, v, "true" if sign[v] else "false") for v in sorted(m)))
        for k, m in sorted(comps.items()))


def intended_run(src, dst, window_edges: int) -> List[Tuple[bool, Dict[int, int], Dict[int, bool]]]:
    n = len(src)
    W = window_edges if window_edges > 0 else max(n, 1)
    uf = ParityUnionFind()
    out = []
    for lo in range(0, n, W):
        for i in range(lo, min(lo + W, n)):
            uf.union(int(src[i]), int(dst[i]))
        out.append(uf.emission())
    return out


def bfs_bipartition(src, dst) -> Tuple[bool, Dict[int, int], Dict[int, bool]]:
    """Independent check: BFS 2-colouring from each component's minimum vertex."""
    adj: Dict[int, List[int]] = {}
    for a, b in zip(np.asarray(src).tolist(), np.asarray(dst).tolist()):
        adj.setdefault(a, [])
        adj.setdefault(b, [])
        if a != b:                             # self-loops only add their vertex (edgeToCandidate)
            adj[a].append(b)
            adj[b].append(a)
    key: Dict[int, int] = {}
    side: Dict[int, int] = {}
    for s in sorted(adj):
        if s in key:
            continue
        key[s], side[s] = s, 0
        q = deque([s])
        while q:
            x = q.popleft()
            for y in adj[x]:
                if y not in key:
                    key[y], side[y] = s, side[x] ^ 1
                    q.append(y)
                elif side[y] == side[x]:
                    return False, {}, {}
    return True, key, {v: side[v] == 0 for v in key}
