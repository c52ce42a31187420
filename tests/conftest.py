"""pytest configuration: markers, import paths, shared fixtures.

`-m "not gpu"` runs the oracle-vs-golden tests, host-logic tests and the C-ABI load/export
checks on any machine; `-m gpu` runs the parity tests through libfmcw.so on an MI355X.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "fpga-fmcw-radar-processor_amd"
GOLDEN = REPO / "tests" / "golden"
for p in (PKG, REPO / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libfmcw.so")
    config.addinivalue_line("markers", "slow: large sizes")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def lib_built():
    from fmcw import _lib
    if not _lib.LIB_PATH.exists():
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build() / make -C {PKG}")
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(lib_built):
    """The GPU tests require the native library AND a device; they never skip to a fallback."""
    from fmcw import _lib
    n = _lib.device_count()
    if n < 1:
        pytest.fail("no HIP device visible to libfmcw.so (GPU tests must run on an MI355X)")
    return n


def rel_err(a, b):
    """max |a - b| / max |b| (per-frame FFT tolerance of the north star)."""
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-30))
