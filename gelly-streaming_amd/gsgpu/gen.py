"""Synthetic edge streams generated on the device (definition: oracle/gen.c header)."""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

from ._abi import call

RMAT_ABC = (0.57, 0.19, 0.19)        # Graph500 (a, b, c); d = 0.05


def rmat_thresholds(a: float, b: float, c: float) -> Tuple[int, int, int]:
    return int(a * 2 ** 32), int(b * 2 ** 32), int(c * 2 ** 32)


def _stream(stream) -> Optional[int]:
    if stream is None:
        import torch
        return int(torch.cuda.current_stream().cuda_stream)
    return stream if isinstance(stream, int) else int(stream.cuda_stream)


def rmat(src, dst, first: int, scale: int, seed: int, scramble: bool = True,
         abc=RMAT_ABC, stream=None) -> None:
    """Fill device tensors src/dst (int32 or int64) with edges [first, first+n) of the RMAT stream."""
    import torch
    assert src.is_cuda and dst.is_cuda and src.numel() == dst.numel()
    bits = 32 if src.dtype == torch.int32 else 64
    ta, tb, tc = rmat_thresholds(*abc)
    call("gs_gen_rmat", ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), bits,
         int(first), src.numel(), int(scale), int(seed), ta, tb, tc, 1 if scramble else 0, _stream(stream))


def erdos_renyi(src, dst, first: int, nv: int, seed: int, stream=None) -> None:
    import torch
    assert src.is_cuda and dst.is_cuda and src.numel() == dst.numel()
    bits = 32 if src.dtype == torch.int32 else 64
    call("gs_gen_er", ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), bits,
         int(first), src.numel(), int(nv), int(seed), _stream(stream))
