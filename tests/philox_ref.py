"""Host restatement of the framework's perf-mode device RNG (common.hpp
pair_normals, pf_kernels.inl resample_offset): Philox-4x32-10 and
Philox-2x32-10 (Random123's round constants and key schedule) in NumPy uint64
arithmetic, Box-Muller on 32-bit uniforms with the C library's log / sqrt /
cos / sin.  Test infrastructure: shared by tests/test_gpu_philox.py and the
bench-path lockstep (tests/test_gpu_run_oracle.py)."""
import numpy as np

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


def resample_u(stepno, seed):
    """pf_kernels.inl resample_offset with no host offset: the rand() of
    particle_filter.py:214 drawn from Philox-4x32-10 (counter (0, 0,
    kStreamResample = 2, stepno), key seed) as a 53-bit uniform; the device's
    offset is this value times NP_RECIP."""
    x, y, _, _ = philox4x32((np.uint64(0), np.uint64(0), np.uint64(2), np.uint64(stepno)),
                            seed & 0xFFFFFFFF, seed >> 32)
    m = (int(x) >> 5) * (1 << 26) + (int(y) >> 6)
    return float(m) * 2.0 ** -53
