"""CPU: the C-ABI library builds, loads and exports every symbol include/gsgpu.h declares;
calls that need no device validate their arguments; without a GPU the library fails loudly."""
import ctypes
import os
import re
import subprocess

import pytest

import gsgpu
from gsgpu import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsgpu.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(gs_\w+)\s*\(", txt, re.M)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(_abi.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _abi.LIB_PATH]).decode()
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in header_functions() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version():
    L = gsgpu.lib()
    assert L.gs_version() == 2
    for s in _abi.EXPORTED_SYMBOLS:
        assert hasattr(L, s)


def test_config_validation_without_device():
    L = gsgpu.lib()
    h = ctypes.c_void_p()
    cfg = _abi.GsCcConfig(ctypes.sizeof(_abi.GsCcConfig) + 4, 32, 100, 0, 0, 0)
    assert L.gs_cc_create(ctypes.byref(h), ctypes.byref(cfg)) == _abi.GS_ERR_INVALID
    assert b"struct_size" in L.gs_last_error()
    cfg = _abi.GsCcConfig(ctypes.sizeof(_abi.GsCcConfig), 16, 100, 0, 0, 0)
    assert L.gs_cc_create(ctypes.byref(h), ctypes.byref(cfg)) == _abi.GS_ERR_INVALID
    cfg = _abi.GsCcConfig(ctypes.sizeof(_abi.GsCcConfig), 32, 0, 0, 0, 0)
    assert L.gs_cc_create(ctypes.byref(h), ctypes.byref(cfg)) == _abi.GS_ERR_INVALID
    cfg = _abi.GsCcConfig(ctypes.sizeof(_abi.GsCcConfig), 32, 1 << 33, 0, 0, 0)
    assert L.gs_cc_create(ctypes.byref(h), ctypes.byref(cfg)) == _abi.GS_ERR_INVALID
    assert L.gs_cc_create(None, ctypes.byref(cfg)) == _abi.GS_ERR_INVALID


def test_null_handle_is_rejected():
    L = gsgpu.lib()
    assert L.gs_cc_fold(None, None, None, 0) == _abi.GS_ERR_INVALID
    assert L.gs_cc_close_window(None) == _abi.GS_ERR_INVALID
    assert L.gs_cc_destroy(None) == _abi.GS_OK
    assert L.gs_gen_rmat(None, None, 32, 0, 1, 10, 1, 0, 0, 0, 1, None) == _abi.GS_ERR_INVALID


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(gsgpu.GsError) as ei:
        gsgpu.DisjointSet(1000)
    assert ei.value.code == _abi.GS_ERR_HIP


def test_missing_library_fails_loudly(tmp_path):
    code = ("import os, sys; os.environ['GSGPU_LIB'] = %r; sys.path.insert(0, %r)\n"
            "import gsgpu\n"
            "try:\n    gsgpu.lib()\nexcept gsgpu.GsgpuUnavailable as e:\n    print('UNAVAILABLE')\n"
            % (str(tmp_path / "nope.so"), os.path.join(ROOT, "gelly-streaming_amd")))
    out = subprocess.check_output(["python", "-c", code]).decode()
    assert "UNAVAILABLE" in out
