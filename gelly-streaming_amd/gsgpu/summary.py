"""Device-backed ``DisjointSet`` summary and the ``UpdateCC`` / ``CombineCC`` functions.

Mirrors the reference's hot-path types (paths relative to the reference's
src/main/java/org/apache/flink/graph/streaming/):

* ``DisjointSet``   — summaries/DisjointSet.java:25-150. One libgsgpu handle = one summary,
  held as a dense uint32 parent array in HBM. ``union`` / ``find`` / ``merge`` / ``getMatches``
  / ``toString`` keep the Java names and meaning; ``find`` returns ``None`` for unknown ids like
  the Java method (:67-69). ``getMatches`` returns the canonical vertex -> root map (the roots
  here are always the component minima, see csrc/cc_kernels.hpp).
* ``UpdateCC``      — library/ConnectedComponents.java:83-85 (EdgesFold: ``ds.union(u, v)``),
  with a batched form ``fold_batch`` that is what the streaming operator calls.
* ``CombineCC``     — library/ConnectedComponents.java:116-125 (merge the smaller summary into
  the larger, return the larger).

Buffers: numpy arrays (host) or torch tensors (host or device) of the handle's id width.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _abi
from ._abi import GsCcConfig, call

U64 = ctypes.c_uint64


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


# torch.Tensor and the dtypes a buffer may have, once torch is loaded (the per-call checks below
# run once per window of a per-window caller: config 5's 2^16-edge windows cost ~25 us each)
_TORCH = None


def _torch_kinds():
    global _TORCH
    if _TORCH is None:
        import torch
        _TORCH = (torch.Tensor, (torch.int32, torch.uint32), (torch.int64,))
    return _TORCH


def _buf(x, id_bits: int, name: str):
    """(pointer, keepalive, length) for a 1-D id buffer of the handle's width."""
    if _TORCH is not None and isinstance(x, _TORCH[0]) or _TORCH is None and _is_torch(x):
        tensor, d32, d64 = _torch_kinds()
        if x.dtype not in (d32 if id_bits == 32 else d64):
            raise TypeError("%s: torch dtype %s, expected %s" % (name, x.dtype, (d32 if id_bits == 32 else d64)[0]))
        if not x.is_contiguous():
            raise ValueError("%s: tensor must be contiguous" % name)
        return ctypes.c_void_p(x.data_ptr()), x, x.numel()
    a = np.asarray(x)
    if id_bits == 32:
        if a.dtype not in (np.int32, np.uint32):
            a = a.astype(np.int64)
            if a.size and (a.min() < 0 or a.max() > 0xFFFFFFFE):
                raise ValueError("%s: ids do not fit 32 bits" % name)
            a = a.astype(np.uint32)
    else:
        a = a.astype(np.int64, copy=False)
    a = np.ascontiguousarray(a)
    return a.ctypes.data_as(ctypes.c_void_p), a, a.size


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)        # torch.cuda.Stream


def _cuda_tensors(objs):
    return [o for o in objs if _is_torch(o) and o.is_cuda]


_MODES = {"allgather": _abi.GS_MERGE_ALLGATHER, "gather": _abi.GS_MERGE_GATHER, "tree": _abi.GS_MERGE_TREE,
          "prefilter": _abi.GS_MERGE_PREFILTER}


def _first_cuda_tensor(objs):
    tensor = _torch_kinds()[0] if _TORCH is not None else None
    for o in objs:
        if (isinstance(o, tensor) if tensor is not None else _is_torch(o)) and o.is_cuda:
            return o
    return None


_RAW_STREAM = []                                  # [torch._C._cuda_getCurrentRawStream or None], first use


def _current_raw_stream(t) -> int:
    """torch's current stream on t's device as a raw pointer (torch.cuda.current_stream builds a
    Stream object per call: a few us, the order of a small window's GPU time)."""
    if not _RAW_STREAM:
        import torch
        _RAW_STREAM.append(getattr(torch._C, "_cuda_getCurrentRawStream", None))
    f = _RAW_STREAM[0]
    if f is not None:
        i = t.get_device()                             # (an int: t.device builds a torch.device)
        return int(f(i))
    import torch
    return int(torch.cuda.current_stream(t.device).cuda_stream)


def _as_torch_stream(hs: int, device):
    """The handle's stream as a torch stream object (0: the null stream, which a non-blocking torch
    stream is NOT ordered with, so it gets the event wait like any other)."""
    import torch
    return torch.cuda.ExternalStream(hs, device=device) if hs else torch.cuda.default_stream(device)


class DisjointSet:
    """GPU union-find summary (DisjointSet<K>), K = int32 or int64 vertex ids in [0, capacity);
    ``sparse=True`` (64-bit ids only): ANY Java long ids, at most ``vertex_capacity`` distinct."""

    def __init__(self, vertex_capacity: int, id_bits: int = 64, device: int = 0,
                 track_marks: bool = False, stream=None, staging_edges: int = 0, sparse: bool = False):
        self.id_bits = int(id_bits)
        self.capacity = int(vertex_capacity)
        self.device = int(device)
        self.sparse = bool(sparse)
        flags = (_abi.GS_CC_TRACK_MARKS if track_marks else 0) | (_abi.GS_CC_SPARSE_IDS if sparse else 0)
        cfg = GsCcConfig(ctypes.sizeof(GsCcConfig), self.id_bits, self.capacity, self.device, flags,
                         int(staging_edges))
        h = ctypes.c_void_p()
        call("gs_cc_create", ctypes.byref(h), ctypes.byref(cfg))
        self._h = h
        self.track_marks = bool(track_marks)
        self._epend = []                        # async delta emissions not yet waited for
        if stream is not None:
            self.set_stream(stream)

    # ---- lifetime ----
    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise RuntimeError("DisjointSet is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            _abi.lib().gs_cc_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass

    def reset(self) -> None:
        """Back to ``new DisjointSet<K>()`` (the fold's initial value)."""
        call("gs_cc_reset", self.handle)

    def set_stream(self, stream) -> None:
        call("gs_cc_set_stream", self.handle, _stream_ptr(stream))
        self._hs = None                             # re-read by _stream()

    def _stream(self) -> int:
        """The handle's HIP stream (cached: it changes only through set_stream)."""
        hs = getattr(self, "_hs", None)
        if hs is None:
            s = ctypes.c_void_p()
            call("gs_cc_get_stream", self.handle, ctypes.byref(s))
            hs = self._hs = int(s.value or 0)
        return hs

    def _after_torch(self, *objs) -> None:
        """Device tensors a call reads were produced in torch's stream order: the handle's stream
        waits for torch's current stream first (an event, no host wait). Without it a handle on
        its own stream could read a tensor torch is still writing (e.g. the torch.stack of a
        fold_pairs input; round 4's list-close diagnostic failed that way)."""
        # (per-call host cost matters: config 5 calls this once per 2^16-edge window, ~25 us of work;
        # the handle's stream is cached and torch's current stream read raw, round 6)
        t = _first_cuda_tensor(objs)
        if t is None:
            return
        hs = self._stream()
        if hs == _current_raw_stream(t):                 # same stream: ordered anyway
            return
        import torch
        cur = torch.cuda.current_stream(t.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        _as_torch_stream(hs, t.device).wait_event(ev)

    def _torch_after(self, *objs) -> None:
        """The reverse: torch's current stream waits for what this handle enqueued into device
        tensors without a host wait (async exports)."""
        t = _first_cuda_tensor(objs)
        if t is None:
            return
        hs = self._stream()
        if hs == _current_raw_stream(t):
            return
        import torch
        cur = torch.cuda.current_stream(t.device)
        ev = torch.cuda.Event()
        ev.record(_as_torch_stream(hs, t.device))
        cur.wait_event(ev)

    def sync(self) -> None:
        call("gs_cc_sync", self.handle)

    # ---- DisjointSet.java API ----
    def makeSet(self, e: int) -> None:
        """makeSet (:53-56) for an id not yet in the summary (= union(e, e))."""
        self.union(e, e)

    def union(self, e1: int, e2: int) -> None:
        """union (:92-118) of one pair."""
        self.fold(np.array([e1]), np.array([e2]))

    def find(self, e: int) -> Optional[int]:
        """find (:66-80): root of e, or None if e is not in the summary."""
        if self.sparse:
            r, found = self.find_batch_flags(np.array([e], dtype=np.int64))
            return int(r[0]) if found[0] else None
        r = self.find_batch(np.array([e]))
        return None if int(r[0]) < 0 else int(r[0])

    def find_batch(self, ids) -> np.ndarray:
        p, keep, n = _buf(ids, self.id_bits, "ids")
        out = np.empty(n, dtype=np.uint32 if self.id_bits == 32 else np.int64)
        self._after_torch(keep)
        call("gs_cc_find", self.handle, p, out.ctypes.data_as(ctypes.c_void_p), n)
        return out.view(np.int32).astype(np.int64) if self.id_bits == 32 else out

    def find_batch_flags(self, ids) -> Tuple[np.ndarray, np.ndarray]:
        """(labels, found): found[i] False where ids[i] is not in the summary (null)."""
        p, keep, n = _buf(ids, self.id_bits, "ids")
        out = np.empty(n, dtype=np.uint32 if self.id_bits == 32 else np.int64)
        found = np.empty(n, dtype=np.uint8)
        self._after_torch(keep)
        call("gs_cc_find_flags", self.handle, p, out.ctypes.data_as(ctypes.c_void_p),
             found.ctypes.data_as(ctypes.c_void_p), n)
        lab = out.view(np.int32).astype(np.int64) if self.id_bits == 32 else out
        return lab, found.astype(bool)

    def merge(self, other: "DisjointSet") -> None:
        """merge (:127-131): union every (key, parent) of ``other`` into this summary."""
        call("gs_cc_merge", self.handle, other.handle)

    def getMatches(self) -> Dict[int, int]:
        v, l = self.pairs()
        return dict(zip(v.tolist(), l.tolist()))

    def size(self) -> int:
        """getMatches().size(): number of vertices in the summary."""
        return self.stats()[0]

    __len__ = size

    def toString(self) -> str:
        """``{root=[members...], ...}`` like DisjointSet.toString (:133-150); roots ascending,
        members ascending (the Java HashMap order is unspecified)."""
        v, l = self.pairs()
        comps: Dict[int, List[int]] = {}
        for a, b in zip(v.tolist(), l.tolist()):
            comps.setdefault(b, []).append(a)
        return "{" + ", ".join("%d=[%s]" % (r, ", ".join(map(str, m))) for r, m in sorted(comps.items())) + "}"

    __str__ = toString

    # ---- batched / streaming API ----
    def fold(self, src, dst) -> None:
        """UpdateCC over a batch: union(src[i], dst[i]) for every i."""
        ps, ks, n = _buf(src, self.id_bits, "src")
        pd, kd, m = _buf(dst, self.id_bits, "dst")
        if n != m:
            raise ValueError("src and dst lengths differ (%d, %d)" % (n, m))
        self._after_torch(ks, kd)
        call("gs_cc_fold", self.handle, ps, pd, n)

    def fold_pairs(self, pairs, n: Optional[int] = None, id_bits: Optional[int] = None) -> None:
        """union over interleaved (u, v) pairs; id_bits=32 folds exported partial summaries."""
        bits = self.id_bits if id_bits is None else id_bits
        p, keep, total = _buf(pairs, bits, "pairs")
        cnt = total // 2 if n is None else int(n)
        if cnt * 2 > total:
            raise ValueError("pairs buffer holds %d pairs, %d requested" % (total // 2, cnt))
        self._after_torch(keep)
        call("gs_cc_fold_pairs32" if bits == 32 else "gs_cc_fold_pairs", self.handle, p, cnt)

    def close_window(self) -> None:
        """Merger step: compress so every label is the canonical (min-id) root."""
        call("gs_cc_close_window", self.handle)

    def merge_window(self, comm, mode: str = "allgather") -> None:
        """Multi-GPU CombineCC of this window (gs_cc_merge_window): exchange this rank's partial
        summary over ``comm`` (gsgpu.comm.Comm) and close the window. Needs track_marks=True."""
        from .comm import MODES
        call("gs_cc_merge_window", self.handle, comm.handle, MODES[mode])

    def fold_windows(self, src, dst, window_edges: int, comm=None, mode: str = "allgather") -> int:
        """A batch of count windows in one call (gs_cc_fold_windows): fold each window of
        ``window_edges`` edges, then close it (or merge it over ``comm``). Returns the windows."""
        ps, ks, n = _buf(src, self.id_bits, "src")
        pd, kd, m = _buf(dst, self.id_bits, "dst")
        if n != m:
            raise ValueError("src and dst lengths differ (%d, %d)" % (n, m))
        w = U64()
        self._after_torch(ks, kd)
        call("gs_cc_fold_windows", self.handle, comm.handle if comm is not None else None,
             _MODES[mode], ps, pd, n, int(window_edges), ctypes.byref(w))
        return int(w.value)

    def fold_text(self, text, window_edges: int, chunk_bytes: int = 0, on_window=None) -> Tuple[int, int]:
        """gs_cc_fold_text: edge text (ConnectedComponentsExample's file format) streamed into this
        summary in count windows, each closed; the ids never leave the device. ``text``: bytes /
        bytearray / numpy uint8 (host), a pinned torch uint8 tensor (DMA straight from it) or a CUDA
        uint8 tensor. on_window(w): called after window w's close is enqueued (read its emission
        there). Returns (edges, windows). A rejected line raises GsError (code GS_ERR_INVALID) with
        ``.edges`` = its 0-based line number (every line before it was folded)."""
        keep = text
        if _is_torch(text):
            p, n = ctypes.c_void_p(text.data_ptr()), text.numel() * text.element_size()
            self._after_torch(text)
        elif isinstance(text, (bytes, bytearray, memoryview)):
            keep = np.frombuffer(text, dtype=np.uint8)
            p, n = keep.ctypes.data_as(ctypes.c_void_p), keep.size
        else:
            keep = np.ascontiguousarray(text, dtype=np.uint8)
            p, n = keep.ctypes.data_as(ctypes.c_void_p), keep.size
        return self._fold_stream("gs_cc_fold_text", (p, n), window_edges, chunk_bytes, on_window)

    def fold_file(self, path: str, window_edges: int, chunk_bytes: int = 0, on_window=None) -> Tuple[int, int]:
        """gs_cc_fold_file: as fold_text, the text read from ``path`` chunk by chunk into pinned
        staging (the whole file never sits in host memory)."""
        return self._fold_stream("gs_cc_fold_file", (str(path).encode(),), window_edges, chunk_bytes, on_window)

    _WINDOW_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64)

    def _fold_stream(self, name, src_args, window_edges, chunk_bytes, on_window):
        errs = []

        def cb(_ctx, w):
            try:
                on_window(int(w))
            except Exception as e:  # an exception cannot cross the C frame: re-raised after the call
                errs.append(e)
        fn = self._WINDOW_FN(cb) if on_window is not None else ctypes.cast(None, self._WINDOW_FN)
        edges, wins = U64(), U64()
        rc = getattr(_abi.lib(), name)(self.handle, *src_args, int(window_edges), int(chunk_bytes), fn, None,
                                       ctypes.byref(edges), ctypes.byref(wins))
        if errs:
            raise errs[0]
        if rc != _abi.GS_OK:
            msg = _abi.lib().gs_last_error()
            e = _abi.GsError(rc, name, msg.decode() if msg else "")
            e.edges, e.windows = int(edges.value), int(wins.value)
            raise e
        return int(edges.value), int(wins.value)

    def stats(self) -> Tuple[int, int]:
        nv, nc = U64(), U64()
        call("gs_cc_stats", self.handle, ctypes.byref(nv), ctypes.byref(nc))
        return int(nv.value), int(nc.value)

    def num_components(self) -> int:
        return self.stats()[1]

    def checksum(self) -> Tuple[int, int, int]:
        s, nv, nc = U64(), U64(), U64()
        call("gs_cc_checksum", self.handle, ctypes.byref(s), ctypes.byref(nv), ctypes.byref(nc))
        return int(s.value), int(nv.value), int(nc.value)

    def dense(self, n: Optional[int] = None, out=None):
        """labels[v] for v < n (default capacity): canonical label or -1."""
        n = self.capacity if n is None else int(n)
        if out is None:
            out = np.empty(n, dtype=np.int32 if self.id_bits == 32 else np.int64)
        p, keep, m = _buf(out, self.id_bits, "labels")
        self._after_torch(keep)
        call("gs_cc_emit_dense", self.handle, p, m)
        return out

    def pairs(self) -> Tuple[np.ndarray, np.ndarray]:
        """(vertices, labels) of every vertex in the summary, sorted by vertex."""
        cnt = U64()
        nv = self.stats()[0]
        dt = np.int32 if self.id_bits == 32 else np.int64
        v = np.empty(max(nv, 1), dtype=dt)
        l = np.empty(max(nv, 1), dtype=dt)
        call("gs_cc_emit_pairs", self.handle, v.ctypes.data_as(ctypes.c_void_p),
             l.ctypes.data_as(ctypes.c_void_p), nv, ctypes.byref(cnt))
        return v[:cnt.value].astype(np.int64), l[:cnt.value].astype(np.int64)

    def delta(self, vertices=None, labels=None) -> Tuple[np.ndarray, np.ndarray]:
        """gs_cc_emit_delta: the (vertex, label) pairs new or changed since the previous delta,
        sorted by vertex (the first delta is the whole emission). Into the given buffers (host
        numpy or device tensors, id_bits wide) if passed, else into fresh numpy arrays sized from
        the summary. Returns views of the filled prefix."""
        dt = np.int32 if self.id_bits == 32 else np.int64
        if vertices is None:
            n = max(self.stats()[0], 1)
            vertices, labels = np.empty(n, dtype=dt), np.empty(n, dtype=dt)
        pv, kv, cap = _buf(vertices, self.id_bits, "vertices")
        pl, kl, cap2 = _buf(labels, self.id_bits, "labels")
        cnt = U64()
        self._after_torch(kv, kl)
        call("gs_cc_emit_delta", self.handle, pv, pl, min(cap, cap2), ctypes.byref(cnt))
        return vertices[:cnt.value], labels[:cnt.value]

    def delta_async(self, vertices, labels) -> None:
        """gs_cc_emit_delta_async: this window's delta, enqueued only, into device tensors or PINNED
        host tensors (id_bits wide); the next fold may be enqueued at once. The buffers are valid
        after emit_wait() returns their entry."""
        pv, kv, cap = _buf(vertices, self.id_bits, "vertices")
        pl, kl, cap2 = _buf(labels, self.id_bits, "labels")
        cnt = U64()
        self._after_torch(kv, kl)
        call("gs_cc_emit_delta_async", self.handle, pv, pl, min(cap, cap2), ctypes.byref(cnt))
        self._epend.append((vertices, labels, cnt, kv, kl))

    def emit_wait(self, keep: int = 0):
        """gs_cc_emit_wait: completes async emissions, oldest first, until at most `keep` are
        pending; returns [(vertices_prefix, labels_prefix), ...] of the completed ones."""
        n_done = max(len(self._epend) - keep, 0)
        done, self._epend = self._epend[:n_done], self._epend[n_done:]
        call("gs_cc_emit_wait", self.handle, keep)
        return [(v[:c.value], l[:c.value]) for v, l, c, _, _ in done]

    # ---- checkpoint / resume (Merger implements ListCheckpointed, SummaryAggregation.java:127-135) ----
    def snapshot(self) -> Tuple[np.ndarray, np.ndarray]:
        """The summary as its canonical (vertex, label) pairs, sorted by vertex: everything the
        reference's snapshotState serialises (the DisjointSet's matches, here canonicalised)."""
        return self.pairs()

    def restore(self, vertices, labels) -> None:
        """restoreState: this summary becomes the snapshotted one (reset, then union(v, label)
        for every pair: the same vertex set and components, hence the same emission)."""
        v = np.asarray(vertices, dtype=np.int64)
        l = np.asarray(labels, dtype=np.int64)
        if v.shape != l.shape:
            raise ValueError("restore: %d vertices, %d labels" % (v.size, l.size))
        self.reset()
        if v.size == 0:
            return
        inter = np.empty(2 * v.size, dtype=np.int64)
        inter[0::2] = v
        inter[1::2] = l
        self.fold_pairs(inter, v.size)
        self.close_window()

    def labels_device_ptr(self) -> int:
        p = ctypes.c_void_p()
        call("gs_cc_labels_device", self.handle, ctypes.byref(p))
        return int(p.value or 0)

    def export_marks(self, out, cap_pairs: Optional[int] = None) -> int:
        """Write this window's partial-summary pairs into ``out`` — uint32 (vertex, root) interleaved,
        or int64 (id, root id) for a sparse-id summary; returns the number of pairs written."""
        p, keep, total = _buf(out, 64 if self.sparse else 32, "out")
        cap = total // 2 if cap_pairs is None else int(cap_pairs)
        n = U64()
        self._after_torch(keep)
        call("gs_cc_export_marks", self.handle, p, cap, ctypes.byref(n))
        return int(n.value)

    def export_marks_async(self, out, count) -> None:
        """export_marks enqueued on the stream; the pair count lands in the device int64 tensor
        ``count`` (one element), no host sync."""
        p, keep, total = _buf(out, 32, "out")
        self._after_torch(keep, count)
        call("gs_cc_export_marks_async", self.handle, p, total // 2, ctypes.c_void_p(count.data_ptr()))
        self._torch_after(keep, count)

    def filter_edges(self, src, dst, out) -> int:
        """The giant pre-filter alone (gs_cc_filter_edges): the edges of (src, dst) that survive this
        summary's giant filter, as uint32 (u, v) pairs into the int32 device tensor ``out``
        (>= 2 x len(src) elements); returns their number. Nothing is folded."""
        ps, ks, n = _buf(src, self.id_bits, "src")
        pd, kd, m = _buf(dst, self.id_bits, "dst")
        if n != m:
            raise ValueError("src and dst differ in length")
        po, ko, total = _buf(out, 32, "out")
        self._after_torch(ks, kd, ko)
        cnt = ctypes.c_uint64()
        call("gs_cc_filter_edges", self.handle, ps, pd, n, po, total // 2, ctypes.byref(cnt))
        return int(cnt.value)

    def set_marking(self, on: bool) -> None:
        """Pause / resume marking (GS_CC_TRACK_MARKS): folds while paused are not exported."""
        call("gs_cc_set_marking", self.handle, 1 if on else 0)

    # ---- instrumentation ----
    def timing(self, enable) -> None:
        """True / False, or GS_TIMING_MASK | (1 << GS_K_*) ...: time only those kernels."""
        call("gs_cc_timing", self.handle, int(enable) if not isinstance(enable, bool) else (1 if enable else 0))

    def kernel_time(self, kernel: int) -> Tuple[float, int]:
        ms, n = ctypes.c_double(), U64()
        call("gs_cc_kernel_time", self.handle, int(kernel), ctypes.byref(ms), ctypes.byref(n))
        return float(ms.value), int(n.value)

    def kernel_units(self, kernel: int) -> int:
        """Edges (folds, merges) or vertices (closes) the timed launches of that class processed."""
        u = U64()
        call("gs_cc_kernel_units", self.handle, int(kernel), ctypes.byref(u))
        return int(u.value)

    def fold_time(self) -> Tuple[float, int]:
        """(ms, launches) of every UpdateCC launch: k_fold (young / plain) + the steady k_fold_ring."""
        a, na = self.kernel_time(_abi.GS_K_FOLD)
        b, nb = self.kernel_time(_abi.GS_K_RING)
        return a + b, na + nb


def combine_cc(s1: DisjointSet, s2: DisjointSet) -> DisjointSet:
    """CombineCC.reduce (ConnectedComponents.java:116-125) on two device summaries."""
    out = ctypes.c_void_p()
    call("gs_cc_combine", s1.handle, s2.handle, ctypes.byref(out))
    return s1 if out.value == s1.handle.value else s2


class UpdateCC:
    """EdgesFold<K, NullValue, DisjointSet<K>> (ConnectedComponents.java:70-86)."""

    def foldEdges(self, ds: DisjointSet, vertex: int, vertex2: int, edgeValue=None) -> DisjointSet:
        ds.union(vertex, vertex2)
        return ds

    def fold_batch(self, ds: DisjointSet, src, dst) -> DisjointSet:
        ds.fold(src, dst)
        return ds


class CombineCC:
    """ReduceFunction<DisjointSet<K>> (ConnectedComponents.java:95-126)."""

    def reduce(self, s1: DisjointSet, s2: DisjointSet) -> DisjointSet:
        return combine_cc(s1, s2)
