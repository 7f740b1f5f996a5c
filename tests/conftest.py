import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# In-process tests run the library's production defaults. Fold variants (the ring fold and warm
# set at small sizes, forced young splits, ...) are named subprocess cases in
# tests/test_gpu_variants.py: the library reads its debug variables once per process.
for p in (ROOT, os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
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
