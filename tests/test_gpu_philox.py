"""The perf-mode device RNG (motion noise of the bench path) against a host
restatement: Philox-4x32-10 and Philox-2x32-10 (Random123's round constants
and key schedule, restated here with NumPy uint64 arithmetic), then Box-Muller
on 32-bit uniforms in float64 with the C library's log / sqrt / cos / sin.

This stream is the framework's own (the reference draws from np.random, which
the device reproduces bit-exactly in noise="mt19937" mode, test_gpu_rng.py);
the bar is the Box-Muller transcendentals' accuracy: every normal within
2e-15 (|g| + 1) of the host's, the 32-bit words bit-exact by construction
(a word error would show as an O(1) difference).  Also: first and second
moments of 2^20 x 6 normals.
"""
import ctypes as C

import numpy as np
import pytest

from philox_ref import host_pair_normals

pytestmark = pytest.mark.gpu


def _device(p0, count, rstep, seed):
    from slamhip import _lib
    lib = _lib.load()
    out = np.empty((count, 6))
    rc = lib.slam_debug_pair_normals(0, p0, count, rstep, seed,
                                     out.ctypes.data_as(C.POINTER(C.c_double)))
    assert rc == 0
    return out


@pytest.mark.parametrize("p0,rstep,seed", [(0, 0, 0), (1 << 19, 7, 3), ((1 << 33) + 5, 123456, 0xDEADBEEF12345678)])
def test_device_normals_match_host_restatement(p0, rstep, seed):
    count = 1 << 16
    dev = _device(p0, count, rstep, seed)
    host, rad = host_pair_normals(np.arange(p0, p0 + count, dtype=np.uint64), rstep, seed)
    err = np.abs(dev - host)
    assert np.all(err <= 2e-15 * (rad + 1.0)), float((err / (rad + 1.0)).max())


def test_device_normals_moments():
    dev = _device(0, 1 << 20, 1, 7).ravel()
    n = dev.size
    assert abs(dev.mean()) < 5.0 / np.sqrt(n)
    assert abs(dev.var() - 1.0) < 5.0 * np.sqrt(2.0 / n)
    assert np.abs(dev).max() < 6.7                  # 32-bit radius: |g| <= sqrt(64 ln 2)
