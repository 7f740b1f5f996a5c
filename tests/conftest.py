import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# The warm set (libgsgpu, cc_kernels.hpp) is on only for ids >= 2^25 in production; the parity
# tests run it from 2^20 ids (read once by the library at its first summary), so every per-window
# oracle comparison of a >= 2^20-id stream goes through it. tests/test_gpu_parity.py runs the
# production default (and GSGPU_WARM=0) in subprocesses.
os.environ.setdefault("GSGPU_WARM_MIN_BITS", "20")
# Likewise the steady ring fold (LDS hot set) runs from 2^20 ids in tests (production: from 2^25;
# the auto choice is run by the fold-variant subprocesses).
os.environ.setdefault("GSGPU_FOLD_MODE", "ring")
for p in (ROOT, os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _oracle_built():
    lib = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")], stdout=subprocess.DEVNULL)
    yield


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import coracle
    return coracle()
