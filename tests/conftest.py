"""Shared pytest setup: markers, import paths, golden-fixture loader."""
import os
import sys

import numpy as np
import pytest

# device kernel arguments, as bench.py (set before anything initialises HIP; llampc itself
# leaves the process environment alone)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "lla-mpc_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests proper")


def golden(name):
    """Load a committed fixture written by tests/golden/gen_golden.py (data only)."""
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold():
    return golden
