"""Shared pytest setup.

Markers: `gpu` — needs an MI355X (run with `-m gpu` on the GPU box).
Everything unmarked runs on the CPU-only container.
"""
import os
import sys

import pytest

# torch (device-buffer plumbing in the GPU tests) must bind its HIP runtime
# before the native library is loaded, so both share one runtime instance.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD MI355X GPU")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # oracle/oracle.py (test infrastructure)
    o.lib()
    return o


@pytest.fixture(scope="session")
def aqz():
    import aqz_pkg
    return aqz_pkg.load()
