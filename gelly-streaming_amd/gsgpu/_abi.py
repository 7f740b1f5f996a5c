"""ctypes binding of libgsgpu.so (C ABI: include/gsgpu.h).

The library is built in-tree (``make -C gelly-streaming_amd``) into ``gsgpu/lib/libgsgpu.so``.
There is no fallback: if the library is missing or cannot be loaded, every entry point raises
``GsgpuUnavailable`` — the HIP path is the only implementation.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSGPU_LIB", os.path.join(HERE, "lib", "libgsgpu.so"))

GS_OK = 0
GS_ERR_INVALID = -1
GS_ERR_HIP = -2
GS_ERR_RANGE = -3
GS_ERR_NOMEM = -4
GS_ERR_STATE = -5
GS_ERR_UNSUPPORTED = -6
GS_ERR_CAPACITY = -7
GS_ERR_COMM = -8

GS_CC_TRACK_MARKS = 1
GS_CC_SPARSE_IDS = 2
GS_BIP_REFERENCE_LITERAL = 1

GS_K_FOLD, GS_K_COMPRESS, GS_K_MERGE, GS_K_EXPORT, GS_K_RING = 0, 1, 2, 3, 4
GS_MERGE_ALLGATHER, GS_MERGE_GATHER, GS_MERGE_TREE, GS_MERGE_PREFILTER = 0, 1, 2, 3
GS_TIMING_MASK = 0x100

_ERRNAMES = {GS_ERR_INVALID: "INVALID", GS_ERR_HIP: "HIP", GS_ERR_RANGE: "RANGE",
             GS_ERR_NOMEM: "NOMEM", GS_ERR_STATE: "STATE", GS_ERR_UNSUPPORTED: "UNSUPPORTED",
             GS_ERR_CAPACITY: "CAPACITY", GS_ERR_COMM: "COMM"}

# every symbol include/gsgpu.h declares (tests check the library exports all of them)
EXPORTED_SYMBOLS = (
    "gs_cc_create", "gs_cc_destroy", "gs_cc_reset", "gs_cc_set_stream", "gs_cc_get_stream",
    "gs_cc_sync", "gs_cc_fold", "gs_cc_fold_pairs", "gs_cc_merge", "gs_cc_combine",
    "gs_cc_close_window", "gs_cc_stats", "gs_cc_emit_dense", "gs_cc_emit_pairs", "gs_cc_emit_delta",
    "gs_cc_emit_delta_async", "gs_cc_emit_wait",
    "gs_cc_checksum", "gs_cc_find", "gs_cc_find_flags", "gs_cc_labels_device", "gs_cc_export_marks",
    "gs_cc_fold_pairs32", "gs_cc_export_marks_async", "gs_cc_filter_edges", "gs_cc_set_marking", "gs_cc_timing", "gs_cc_kernel_time", "gs_cc_kernel_units", "gs_gen_rmat", "gs_gen_er", "gs_parse_edges",
    "gs_cc_fold_text", "gs_cc_fold_file",
    "gs_bip_create", "gs_bip_destroy", "gs_bip_reset", "gs_bip_set_stream", "gs_bip_sync", "gs_bip_fold",
    "gs_bip_fold_pairs", "gs_bip_merge", "gs_bip_close_window", "gs_bip_status", "gs_bip_checksum",
    "gs_bip_emit_pairs", "gs_bip_create_ex", "gs_bip_restore",
    "gs_comm_unique_id", "gs_comm_create", "gs_comm_create_local", "gs_comm_destroy", "gs_comm_info",
    "gs_cc_merge_window", "gs_cc_fold_windows",
    "gs_last_error", "gs_version",
)


def lib_source_sha() -> str:
    """sha256 over the library's kernel and boundary sources (csrc/*.hip, csrc/*.hpp, the header):
    committed profiles carry it, so a number measured on other kernels is recognised as stale."""
    import glob
    import hashlib
    pkg = os.path.dirname(HERE)
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.hpp")))
    files.append(os.path.join(os.path.dirname(pkg), "include", "gsgpu.h"))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


class GsgpuUnavailable(RuntimeError):
    """libgsgpu.so is not built or cannot be loaded."""


class GsError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__("%s failed: GS_ERR_%s (%d): %s" % (where, _ERRNAMES.get(code, "?"), code, msg))
        self.code = code


class GsCcConfig(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("id_bits", ctypes.c_uint32),
                ("vertex_capacity", ctypes.c_uint64), ("device", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("staging_edges", ctypes.c_uint64)]


_LIB: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise GsgpuUnavailable("libgsgpu.so not found at %s — build it with `make -C gelly-streaming_amd` "
                               "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
    # One HIP runtime per process: torch's bundled ROCm libraries ask for "libamdhip64.so" (no
    # version), libgsgpu.so for "libamdhip64.so.7". Loaded after torch, libgsgpu binds to torch's
    # runtime (its soname IS libamdhip64.so.7, likewise librccl.so.1); loaded first, it would pull
    # /opt/rocm's and torch would then load a second runtime next to it (two HSA teardowns at
    # exit: "double free or corruption"). So torch, when importable, is loaded first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    try:
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        raise GsgpuUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
    P = ctypes.POINTER
    sig = {
        "gs_cc_create": [P(vp), P(GsCcConfig)],
        "gs_cc_destroy": [vp],
        "gs_cc_reset": [vp],
        "gs_cc_set_stream": [vp, vp],
        "gs_cc_get_stream": [vp, P(vp)],
        "gs_cc_sync": [vp],
        "gs_cc_fold": [vp, vp, vp, u64],
        "gs_cc_fold_pairs": [vp, vp, u64],
        "gs_cc_fold_pairs32": [vp, vp, u64],
        "gs_cc_set_marking": [vp, ctypes.c_int],
        "gs_cc_export_marks_async": [vp, vp, u64, vp],
        "gs_cc_filter_edges": [vp, vp, vp, u64, vp, u64, P(u64)],
        "gs_cc_merge": [vp, vp],
        "gs_cc_combine": [vp, vp, P(vp)],
        "gs_cc_close_window": [vp],
        "gs_cc_stats": [vp, P(u64), P(u64)],
        "gs_cc_emit_dense": [vp, vp, u64],
        "gs_cc_emit_pairs": [vp, vp, vp, u64, P(u64)],
        "gs_cc_emit_delta": [vp, vp, vp, u64, P(u64)],
        "gs_cc_emit_delta_async": [vp, vp, vp, u64, P(u64)],
        "gs_cc_emit_wait": [vp, ctypes.c_uint32],
        "gs_cc_checksum": [vp, P(u64), P(u64), P(u64)],
        "gs_cc_find": [vp, vp, vp, u64],
        "gs_cc_find_flags": [vp, vp, vp, vp, u64],
        "gs_cc_labels_device": [vp, P(vp)],
        "gs_cc_export_marks": [vp, vp, u64, P(u64)],
        "gs_cc_timing": [vp, i32],
        "gs_cc_kernel_time": [vp, i32, P(ctypes.c_double), P(u64)],
        "gs_cc_kernel_units": [vp, i32, P(u64)],
        "gs_gen_rmat": [vp, vp, u32, u64, u64, i32, u64, u32, u32, u32, i32, vp],
        "gs_gen_er": [vp, vp, u32, u64, u64, u64, u64, vp],
        "gs_parse_edges": [vp, u64, u32, vp, vp, u64, P(u64), i32, vp],
        "gs_cc_fold_text": [vp, vp, u64, u64, u64, ctypes.CFUNCTYPE(None, vp, u64), vp, P(u64), P(u64)],
        "gs_cc_fold_file": [vp, ctypes.c_char_p, u64, u64, ctypes.CFUNCTYPE(None, vp, u64), vp, P(u64), P(u64)],
        "gs_bip_create": [P(vp), u64, u32, i32],
        "gs_bip_create_ex": [P(vp), u64, u32, i32, u32, u64],
        "gs_bip_destroy": [vp],
        "gs_bip_reset": [vp],
        "gs_bip_set_stream": [vp, vp],
        "gs_bip_sync": [vp],
        "gs_bip_fold": [vp, vp, vp, u64],
        "gs_bip_fold_pairs": [vp, vp, u64],
        "gs_bip_merge": [vp, vp],
        "gs_bip_close_window": [vp],
        "gs_bip_status": [vp, P(i32), P(u64), P(u64)],
        "gs_bip_checksum": [vp, P(u64), P(i32), P(u64), P(u64)],
        "gs_bip_emit_pairs": [vp, vp, vp, vp, u64, P(u64)],
        "gs_bip_restore": [vp, i32, vp, vp, vp, u64],
        "gs_comm_unique_id": [vp, u64],
        "gs_comm_create": [P(vp), vp, i32, i32, i32],
        "gs_comm_create_local": [P(vp), i32, i32],
        "gs_comm_destroy": [vp],
        "gs_comm_info": [vp, P(i32), P(i32), P(u64), P(u64), P(u64), P(u64)],
        "gs_cc_merge_window": [vp, vp, i32],
        "gs_cc_fold_windows": [vp, vp, i32, vp, vp, u64, u64, P(u64)],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = i32
    L.gs_last_error.argtypes = []
    L.gs_last_error.restype = ctypes.c_char_p
    L.gs_version.argtypes = []
    L.gs_version.restype = i32
    _LIB = L
    return L


_FN = {}                                          # name -> ctypes function (a per-call getattr costs)


def call(name: str, *args) -> None:
    f = _FN.get(name)
    if f is None:
        f = _FN[name] = getattr(lib(), name)
    rc = f(*args)
    if rc != GS_OK:
        msg = lib().gs_last_error()
        raise GsError(rc, name, msg.decode() if msg else "")


def available() -> bool:
    try:
        lib()
        return True
    except GsgpuUnavailable:
        return False
