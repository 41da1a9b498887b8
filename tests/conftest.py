import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "coconut-rust_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def oracle_lib():
    """The C oracle (test infrastructure only), built on demand.  CC_ORACLE_SAN=1: the same entry points
    run in the ASan/UBSan build (tests/san_oracle.py; tests/test_sanitizers.py sets it)."""
    import ctypes
    if os.environ.get("CC_ORACLE_SAN") == "1":
        from san_oracle import SanOracle
        return SanOracle()
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle", "c")])
    return ctypes.CDLL(so)


@pytest.fixture(scope="session")
def oc():
    return oracle_lib()


def host_threads():
    """Worker threads for CPU-side helpers: the GPU box grants ~16 cores per GPU (OMP_NUM_THREADS)."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(n or (os.cpu_count() or 8), 16))
