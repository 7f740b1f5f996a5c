"""Edge-file ingestion on the device (gs_parse_edges): the text format and error behaviour of
ConnectedComponentsExample's file input (example/ConnectedComponentsExample.java:108-119)."""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from ._abi import GsError, call


def parse_edges(data: bytes, id_bits: int = 64, device: int = 0, out=None) -> Tuple[np.ndarray, np.ndarray]:
    """Parse edge text -> (src, dst) host arrays (int64 or int32)."""
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


__all__ = ["parse_edges", "read_edge_file", "GsError"]
