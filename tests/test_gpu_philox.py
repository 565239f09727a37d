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

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)


def _u32(x):
    return np.asarray(x, dtype=np.uint64) & M32


def _mulhilo(a, b):
    p = _u32(a) * np.uint64(b)
    return p >> np.uint64(32), p & M32


def philox4x32(c, k0, k1):
    x, y, z, w = [_u32(v) for v in c]
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        hi0, lo0 = _mulhilo(x, 0xD2511F53)
        hi1, lo1 = _mulhilo(z, 0xCD9E8D57)
        x, y, z, w = hi1 ^ y ^ k0, lo1, hi0 ^ w ^ k1, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return x, y, z, w


def philox2x32(c0, c1, k):
    c0, c1, k = _u32(c0), _u32(c1), np.uint64(k)
    for _ in range(10):
        hi, lo = _mulhilo(c0, 0xD256D193)
        c0, c1 = hi ^ k ^ c1, lo
        k = (k + np.uint64(0x9E3779B9)) & M32
    return c0, c1


def bm_pair(a, b):
    rad = np.sqrt(-2.0 * np.log((a.astype(np.float64) + 1.0) * 2.0 ** -32))
    ang = 2.0 * np.pi * ((b.astype(np.float64) + 1.0) * 2.0 ** -32)
    return rad * np.cos(ang), rad * np.sin(ang), rad


def host_pair_normals(p, rstep, seed):
    """common.hpp pair_normals: Philox-4x32-10 (counter (p, p >> 32, stream 1,
    rstep), key seed) -> pairs A, B; Philox-2x32-10 (counter (p, rstep), key
    seed-lo ^ seed-hi * 0x85EBCA6B ^ 3 * 0x27D4EB2F) -> pair C."""
    p = np.asarray(p, dtype=np.uint64)
    s_lo, s_hi = seed & 0xFFFFFFFF, seed >> 32
    x, y, z, w = philox4x32((p & M32, p >> np.uint64(32), np.full_like(p, 1), np.full_like(p, rstep)),
                            s_lo, s_hi)
    k2 = (s_lo ^ ((s_hi * 0x85EBCA6B) & 0xFFFFFFFF)) ^ ((3 * 0x27D4EB2F) & 0xFFFFFFFF)
    c0, c1 = philox2x32(p & M32, np.full_like(p, rstep), k2)
    ga = bm_pair(x, y)
    gb = bm_pair(z, w)
    gc = bm_pair(c0, c1)
    g = np.stack([ga[0], ga[1], gb[0], gb[1], gc[0], gc[1]], 1)
    rad = np.stack([ga[2], ga[2], gb[2], gb[2], gc[2], gc[2]], 1)
    return g, rad


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
