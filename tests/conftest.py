"""pytest configuration: `gpu` marker (tests that need an MI355X), import paths.

The product modules live flat in `pan-tilt-zoom-slam_amd/` (the reference's `slam_system/` layout, so
`from ptz_slam import PtzSlam` works as under demo_soccer.py); the CPU oracle is the `oracle` package at
the repo root (test infrastructure only)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pan-tilt-zoom-slam_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X) and libptzba.so")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f"golden fixture {name} not generated")
    return np.load(path, allow_pickle=False)


@pytest.fixture(scope="session")
def gpu_available():
    import torch  # noqa: F401  (device visibility only)
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
