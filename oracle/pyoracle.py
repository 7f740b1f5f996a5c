"""TEST INFRASTRUCTURE ONLY — Python access to the CPU oracle (parity checker).

Two things live here:

* ``PyDisjointSet`` — a pure-Python twin of ``summaries/DisjointSet.java`` (reference
  src/main/java/org/apache/flink/graph/streaming/summaries/DisjointSet.java:25-150), used for the
  reference's small known-answer tests and to mint golden fixtures (tests/golden/make_golden.py).
* ``COracle`` — ctypes binding of ``oracle/build/liboracle.so`` (the C restatement in this
  directory), used for larger parity cases and for bench.py's ``cpu_baseline``.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline may import this module.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

MASK64 = (1 << 64) - 1


# --------------------------------------------------------------------------------------------
# pure-Python twin of DisjointSet.java
# --------------------------------------------------------------------------------------------
class PyDisjointSet:
    """DisjointSet<R>: ``matches`` (vertex -> parent) and ``ranks`` (vertex -> rank).

    Follows DisjointSet.java line by line: makeSet :53-56, find :66-80 (recursive full path
    compression; None for unknown ids), union :92-118 (union by rank, tie -> root2 under root1),
    merge :127-131, toString :133-150.
    """

    def __init__(self, elements: Optional[Iterable] = None):
        self.matches: Dict = {}
        self.ranks: Dict = {}
        if elements is not None:                  # DisjointSet(Set<R>) :36-42
            for e in elements:
                self.matches[e] = e
                self.ranks[e] = 0

    def getMatches(self) -> Dict:
        return self.matches

    def makeSet(self, e) -> None:
        self.matches[e] = e
        self.ranks[e] = 0

    def find(self, e):
        if e not in self.matches:
            return None
        # iterative form of the recursion; the final state is identical
        path = []
        x = e
        while self.matches[x] != x:
            path.append(x)
            x = self.matches[x]
        for y in path:
            self.matches[y] = x
        return x

    def union(self, e1, e2) -> None:
        if e1 not in self.matches:
            self.makeSet(e1)
        if e2 not in self.matches:
            self.makeSet(e2)
        root1 = self.find(e1)
        root2 = self.find(e2)
        if root1 == root2:
            return
        dist1 = self.ranks[root1]
        dist2 = self.ranks[root2]
        if dist1 > dist2:
            self.matches[root2] = root1
        elif dist1 < dist2:
            self.matches[root1] = root2
        else:
            self.matches[root2] = root1
            self.ranks[root1] = dist1 + 1

    def merge(self, other: "PyDisjointSet") -> None:
        for k, p in list(other.getMatches().items()):
            self.union(k, p)

    def components(self) -> Dict:
        comps: Dict = {}
        for v in list(self.matches.keys()):
            comps.setdefault(self.find(v), []).append(v)
        return comps

    def toString(self) -> str:
        """Same shape as Java's HashMap.toString of {root=[members...]} (:133-150)."""
        parts = []
        for root, members in self.components().items():
            parts.append("%s=[%s]" % (root, ", ".join(str(m) for m in members)))
        return "{" + ", ".join(parts) + "}"

    def canonical(self) -> Dict:
        """vertex -> minimum vertex id of its component."""
        out = {}
        for members in self.components().values():
            m = min(members)
            for v in members:
                out[v] = m
        return out


def combine_cc(s1: PyDisjointSet, s2: PyDisjointSet) -> PyDisjointSet:
    """CombineCC.reduce (library/ConnectedComponents.java:116-125)."""
    if len(s1.getMatches()) <= len(s2.getMatches()):
        s2.merge(s1)
        return s2
    s1.merge(s2)
    return s1


def py_cc_stream(src: Sequence[int], dst: Sequence[int], window_edges: int, partitions: int
                 ) -> List[Dict]:
    """SummaryBulkAggregation.run + Merger over count-based windows (pipeline.c, same split).

    Returns, per window, the canonical emission {vertex: min-id label}.
    """
    n = len(src)
    W = window_edges if window_edges > 0 else max(n, 1)
    P = max(partitions, 1)
    summary: Optional[PyDisjointSet] = None
    out = []
    for lo in range(0, n, W):
        ln = min(W, n - lo)
        acc = None
        for p in range(P):
            a = lo + (ln * p) // P
            b = lo + (ln * (p + 1)) // P
            if a == b:
                continue
            ds = PyDisjointSet()
            for i in range(a, b):
                ds.union(int(src[i]), int(dst[i]))          # UpdateCC.foldEdges
            acc = ds if acc is None else combine_cc(acc, ds)
        summary = acc if summary is None else combine_cc(acc, summary)
        out.append(summary.canonical())
    return out


# --------------------------------------------------------------------------------------------
# shared emission checksum definition (oracle/disjoint_set.c gso_pair_mix)
# --------------------------------------------------------------------------------------------
def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def _np_splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def dense_checksum(labels: np.ndarray) -> Tuple[int, int, int]:
    """(checksum, n_seen, n_components) of a dense label array (label < 0 == unseen)."""
    lab = np.asarray(labels).astype(np.int64)
    v = np.nonzero(lab >= 0)[0].astype(np.uint64)
    l = lab[lab >= 0].astype(np.uint64)
    mix = _np_splitmix64(v ^ _np_splitmix64(l ^ np.uint64(0xD1B54A32D192ED03)))
    with np.errstate(over="ignore"):
        h = int(np.sum(mix, dtype=np.uint64))
    return h, int(v.size), int(np.count_nonzero(l == v))


def canonical_to_dense(canon: Dict, cap: int) -> np.ndarray:
    out = np.full(cap, -1, dtype=np.int64)
    for v, l in canon.items():
        out[v] = l
    return out


# --------------------------------------------------------------------------------------------
# ctypes binding of the C restatement
# --------------------------------------------------------------------------------------------
EMIT_NONE, EMIT_FLATTEN, EMIT_CHECKSUM, EMIT_DENSE, EMIT_TRACK = 0, 1, 2, 3, 4


class _RunCfg(ctypes.Structure):
    _fields_ = [("window_edges", ctypes.c_uint64), ("partitions", ctypes.c_int),
                ("threads", ctypes.c_int), ("emit_mode", ctypes.c_int),
                ("label_cap", ctypes.c_uint64), ("verify_every", ctypes.c_uint64)]


class _RunStats(ctypes.Structure):
    _fields_ = [("windows", ctypes.c_uint64), ("final_vertices", ctypes.c_uint64),
                ("final_components", ctypes.c_uint64), ("seconds", ctypes.c_double)]


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# RMAT Graph500 probabilities (a, b, c, d) = (0.57, 0.19, 0.19, 0.05) as 32-bit thresholds
RMAT_A, RMAT_B, RMAT_C = 0.57, 0.19, 0.19


def rmat_thresholds(a: float = RMAT_A, b: float = RMAT_B, c: float = RMAT_C) -> Tuple[int, int, int]:
    return int(a * 2 ** 32), int(b * 2 ** 32), int(c * 2 ** 32)


class COracle:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError("oracle library not built: %s (run make -C oracle)" % path)
        L = ctypes.CDLL(path)
        vp, u64, i64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
        L.gso_ds_new.restype = vp
        L.gso_ds_free.argtypes = [vp]
        L.gso_ds_size.argtypes = [vp]; L.gso_ds_size.restype = u64
        L.gso_ds_make_set.argtypes = [vp, i64]
        L.gso_ds_find.argtypes = [vp, i64, ctypes.POINTER(i64)]; L.gso_ds_find.restype = i32
        L.gso_ds_union.argtypes = [vp, i64, i64]
        L.gso_ds_merge.argtypes = [vp, vp]
        L.gso_combine.argtypes = [vp, vp]; L.gso_combine.restype = vp
        L.gso_ds_key_at.argtypes = [vp, u64]; L.gso_ds_key_at.restype = i64
        L.gso_ds_canonical_dense.argtypes = [vp, vp, u64]; L.gso_ds_canonical_dense.restype = u64
        L.gso_cc_run.argtypes = [vp, vp, u64, ctypes.POINTER(_RunCfg), vp, vp, vp, ctypes.POINTER(_RunStats)]
        L.gso_cc_run.restype = i32
        L.gso_cc_run_from.argtypes = [vp, vp, u64, vp, vp, u64, ctypes.POINTER(_RunCfg), vp, vp, vp,
                                      ctypes.POINTER(_RunStats)]
        L.gso_cc_run_from.restype = i32
        L.gso_cc_run_counts.argtypes = [vp, vp, u64, vp, vp, u64, ctypes.POINTER(_RunCfg), vp, vp, vp, vp,
                                        ctypes.POINTER(_RunStats)]
        L.gso_cc_run_counts.restype = i32
        L.gso_gen_rmat.argtypes = [vp, vp, u64, u64, i32, u64, u32, u32, u32, i32]
        L.gso_gen_er.argtypes = [vp, vp, u64, u64, u64, u64]
        L.gso_splitmix64.argtypes = [u64]; L.gso_splitmix64.restype = u64
        L.gso_pair_mix.argtypes = [u64, u64]; L.gso_pair_mix.restype = u64
        L.gso_parse_edges.argtypes = [ctypes.c_char_p, u64, vp, vp, u64]; L.gso_parse_edges.restype = i64
        L.gso_bip_run.argtypes = [vp, vp, u64, u64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double)]
        L.gso_bip_run.restype = ctypes.c_int
        self.L = L

    # ---- BipartitenessCheck (bipartite.c) ----
    def bip_run(self, src, dst, window_edges: int, partitions: int = 1, threads: int = 1):
        """(bipartite, vertices, components, seconds) of the stream through the dataflow."""
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        ok, nv, nc, secs = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
        self.L.gso_bip_run(_p(src), _p(dst), int(src.size), int(window_edges), int(partitions), int(threads),
                           ctypes.byref(ok), ctypes.byref(nv), ctypes.byref(nc), ctypes.byref(secs))
        return bool(ok.value), int(nv.value), int(nc.value), float(secs.value)

    # ---- edge-file input (parse.c) ----
    def parse_edges(self, text: bytes):
        """(src, dst, seconds) as int64 arrays, or (bad line index, None, seconds)."""
        import time
        cap = text.count(b"\n") + 1
        src = np.empty(cap, dtype=np.int64)
        dst = np.empty(cap, dtype=np.int64)
        t0 = time.perf_counter()
        r = int(self.L.gso_parse_edges(text, len(text), _p(src), _p(dst), cap))
        secs = time.perf_counter() - t0
        if r < 0:
            return -r - 1, None, secs
        return src[:r], dst[:r], secs

    # ---- generators ----
    def gen_rmat(self, first: int, n: int, scale: int, seed: int, scramble: bool = True,
                 abc: Tuple[float, float, float] = (RMAT_A, RMAT_B, RMAT_C)):
        src = np.empty(n, dtype=np.int64)
        dst = np.empty(n, dtype=np.int64)
        ta, tb, tc = rmat_thresholds(*abc)
        self.L.gso_gen_rmat(_p(src), _p(dst), first, n, scale, seed, ta, tb, tc, 1 if scramble else 0)
        return src, dst

    def gen_er(self, first: int, n: int, nv: int, seed: int):
        src = np.empty(n, dtype=np.int64)
        dst = np.empty(n, dtype=np.int64)
        self.L.gso_gen_er(_p(src), _p(dst), first, n, nv, seed)
        return src, dst

    # ---- pipeline ----
    def run(self, src: np.ndarray, dst: np.ndarray, window_edges: int, partitions: int = 1,
            threads: int = 1, emit: int = EMIT_CHECKSUM, label_cap: int = 0,
            want_final: bool = False, init=None, verify_every: int = 0):
        """The pipeline over (src, dst); init = (vertices, labels): the Merger restored from that
        snapshot first (untimed), so a run can start in the middle of a stream."""
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        n = int(src.size)
        W = window_edges if window_edges > 0 else max(n, 1)
        nwin = (n + W - 1) // W if n else 0
        cfg = _RunCfg(window_edges, partitions, threads, emit, label_cap, verify_every)
        st = _RunStats()
        sums = np.zeros(max(nwin, 1), dtype=np.uint64)
        counts = np.zeros((max(nwin, 1), 2), dtype=np.uint64)     # per window: (vertices, components)
        labels = np.empty((max(nwin, 1), label_cap), dtype=np.int64) if emit == EMIT_DENSE else None
        final = np.empty(label_cap, dtype=np.int64) if (want_final and label_cap) else None
        iv = il = None
        if init is not None and len(init[0]):
            iv = np.ascontiguousarray(init[0], dtype=np.int64)
            il = np.ascontiguousarray(init[1], dtype=np.int64)
        rc = self.L.gso_cc_run_counts(_p(iv), _p(il), 0 if iv is None else int(iv.size), _p(src), _p(dst), n,
                                      ctypes.byref(cfg), _p(sums), _p(counts), _p(labels), _p(final), ctypes.byref(st))
        if rc == -2:
            raise RuntimeError("gso_cc_run: the incremental emission tracker disagrees with the summary's canonical checksum")
        if rc != 0:
            raise RuntimeError("gso_cc_run failed: %d" % rc)
        return {"windows": int(st.windows), "checksums": sums[:nwin], "counts": counts[:nwin], "labels": labels,
                "final": final, "final_vertices": int(st.final_vertices),
                "final_components": int(st.final_components), "seconds": float(st.seconds)}


_COR: Optional[COracle] = None


def coracle() -> COracle:
    global _COR
    if _COR is None:
        _COR = COracle()
    return _COR


# --------------------------------------------------------------------------------------------
# CPU model of one rank's summary in the multi-GPU tree exchange (tests/gloo_tree.py), for the
# gloo tests: min-root hooking union-find over a dense parent array with per-vertex marks of
# the roots hooked / singletons created since the last export — the same contract as
# gs_cc_export_marks / gs_cc_fold_pairs32 (include/gsgpu.h). Pure restatement, no GPU.
# --------------------------------------------------------------------------------------------
class PyMarkedSummary:
    INV = -1

    def __init__(self, cap: int, track_marks: bool = True):
        self.parent = np.full(cap, -1, dtype=np.int64)
        self.mark = np.zeros(cap, dtype=bool)
        self.track = track_marks

    def _root(self, x: int) -> int:
        p = self.parent
        r = x
        while p[r] != r:
            r = int(p[r])
        while p[x] != r:
            nx = int(p[x]); p[x] = r; x = nx
        return r

    def union(self, u: int, v: int) -> None:
        p = self.parent
        if u == v:
            if p[u] < 0:
                p[u] = u
                if self.track:
                    self.mark[u] = True
            return
        if p[u] < 0:
            p[u] = u
        if p[v] < 0:
            p[v] = v
        ru, rv = self._root(u), self._root(v)
        if ru == rv:
            return
        hi, lo = max(ru, rv), min(ru, rv)
        p[hi] = lo
        if self.track:
            self.mark[hi] = True

    def fold(self, src, dst) -> None:
        for a, b in zip(np.asarray(src).tolist(), np.asarray(dst).tolist()):
            self.union(int(a), int(b))

    def fold_pairs(self, buf, n: int, id_bits: int = 32) -> None:
        a = np.asarray(buf.cpu() if hasattr(buf, "cpu") else buf)[: 2 * n].astype(np.int64)
        self.fold(a[0::2], a[1::2])

    def set_marking(self, on: bool) -> None:
        self.track = bool(on)

    def export_marks(self, buf, cap: int) -> int:
        vs = np.nonzero(self.mark)[0][:cap]
        out = np.empty(2 * len(vs), dtype=np.int32)
        out[0::2] = vs
        out[1::2] = [self._root(int(v)) for v in vs]           # (v, root), as k_export_marks
        self.mark[vs] = False
        if hasattr(buf, "copy_"):
            import torch
            buf[: out.size].copy_(torch.from_numpy(out))
        else:
            buf[: out.size] = out
        return int(len(vs))

    def close_window(self) -> None:
        for v in np.nonzero(self.parent >= 0)[0].tolist():
            self._root(v)

    def dense(self) -> np.ndarray:
        self.close_window()
        return self.parent.copy()
