"""Edge-file ingestion on the device: the text format and error behaviour of
ConnectedComponentsExample's file input (example/ConnectedComponentsExample.java:108-119).

* ``fold_edge_file`` / ``fold_edge_text`` — the streaming path the example's
  ``edges.aggregate(new ConnectedComponents(...))`` (:61) takes: the text goes to the device in
  chunks (pinned, double-buffered H2D), is parsed there into an edge ring and folded straight from
  it, window by window (gs_cc_fold_file / gs_cc_fold_text); the ids never come back to the host.
* ``parse_edges`` / ``read_edge_file`` — the device parser alone (gs_parse_edges), for callers that
  want the ids themselves on the host.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional, Tuple

import numpy as np

from ._abi import GsError, call


def fold_edge_file(summary, path: str, window_edges: int, chunk_bytes: int = 0,
                   on_window: Optional[Callable[[int], None]] = None) -> Tuple[int, int]:
    """Stream the edge file at ``path`` into ``summary`` (a gsgpu.DisjointSet) in count windows of
    ``window_edges`` edges, each closed (the Merger's emission; ``on_window(w)`` after window w).
    Returns (edges, windows). A rejected line raises GsError (GS_ERR_INVALID, ``.edges`` = its
    0-based line number, every line before it folded)."""
    return summary.fold_file(path, window_edges, chunk_bytes=chunk_bytes, on_window=on_window)


def fold_edge_text(summary, text, window_edges: int, chunk_bytes: int = 0,
                   on_window: Optional[Callable[[int], None]] = None) -> Tuple[int, int]:
    """As fold_edge_file, for text already in memory (bytes / numpy uint8 / a pinned or CUDA uint8
    torch tensor)."""
    return summary.fold_text(text, window_edges, chunk_bytes=chunk_bytes, on_window=on_window)


def parse_edges(data: bytes, id_bits: int = 64, device: int = 0, out=None) -> Tuple[np.ndarray, np.ndarray]:
    """Parse edge text on the device -> (src, dst) host arrays (int64)."""
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    n = ctypes.c_uint64()
    dt = np.int64 if id_bits == 64 else np.uint32
    cap = data.count(b"\n") + 1
    src = np.empty(cap, dtype=dt)
    dst = np.empty(cap, dtype=dt)
    call("gs_parse_edges", buf, len(data), id_bits, src.ctypes.data_as(ctypes.c_void_p),
         dst.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n), device, None)
    return src[: n.value].astype(np.int64), dst[: n.value].astype(np.int64)


def read_edge_file(path: str, **kw) -> Tuple[np.ndarray, np.ndarray]:
    with open(path, "rb") as f:
        return parse_edges(f.read(), **kw)


__all__ = ["fold_edge_file", "fold_edge_text", "parse_edges", "read_edge_file", "GsError"]
