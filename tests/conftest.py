"""Shared test setup: import paths, the `gpu` marker and golden-fixture loading."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nerf-experiments_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Deferred encoding rows (generated inside the fused forward) are NaN-filled at allocation, so a
# read of a row before the kernel stored it fails every time instead of returning whatever the
# allocator left there (nerf_amd/kernels.py encode_fwd).
os.environ.setdefault("NERF_POISON_DEFERRED", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and the built HIP library")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
        return cache[name]

    return load


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
