import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-robot_simu_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def heavy_weights(rs, n, zero_frac=0.0):
    """Same generator as tests/golden/make_golden.py (multiplications only)."""
    u = rs.random_sample(n)
    v = rs.random_sample(n)
    w = u * u
    w = w * w
    w = w * w
    w = w * w * v
    if zero_frac > 0:
        w[rs.random_sample(n) < zero_frac] = 0.0
    return w


def stage_weights(tag, n, wseed):
    w = heavy_weights(np.random.RandomState(int(wseed)), n,
                      zero_frac=0.5 if tag in ("r8193", "r1m") else 0.0)
    if tag in ("r8193", "r1m"):
        w[:64] = 0.0
    return w / np.sum(w.reshape(1, n))


def rle_decode(vals, counts):
    return np.repeat(vals.astype(np.int64), counts)
