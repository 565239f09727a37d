"""CPU restatement of NumPy's legacy RandomState stream, in the form the device
computes it (TEST INFRASTRUCTURE ONLY: imported by tests/, never by the
product path).

The reference's noise comes from np.random's global RandomState
(particle_filter.py:152 mvn(0, R, NL), :165 mvn(0, Q, NP), :214 rand();
motion_model.py:46-48).  NumPy (numpy/random/src/mt19937/mt19937.c,
legacy/legacy-distributions.c) draws:
  word    temper(key[pos++]), the key regenerated in place when pos == 624;
  double  ((w0 >> 5) * 67108864.0 + (w1 >> 6)) / 9007199254740992.0;
  gauss   the cached normal if one is held; else x1 = 2d - 1, x2 = 2d - 1 until
          0 < r2 = x1^2 + x2^2 < 1, f = sqrt(-2 log(r2) / r2), cache f x1,
          return f x2 (log: the C library's).
This module restates that as the device pipeline does (rng_api.hip): the
untempered sequence X[n + 624] = X[n + 397] ^ twist(X[n], X[n + 1]) generated
ahead, candidate pairs of four words, the first P accepted pairs, and the state
NumPy leaves behind.  Pinned against RandomState itself in
tests/test_rng_restatement.py (the reference's own dependency, importable here).
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

N, M = 624, 397
MATRIX_A = np.uint32(0x9908B0DF)
UPPER, LOWER = np.uint32(0x80000000), np.uint32(0x7FFFFFFF)

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.log.restype = ctypes.c_double
_libm.log.argtypes = [ctypes.c_double]


def libm_log(x):
    """The C library's log, element by element (what legacy_gauss calls)."""
    return np.array([_libm.log(float(v)) for v in np.ravel(x)])


def _twist(xn, xn1, xm):
    y = (xn & UPPER) | (xn1 & LOWER)
    return xm ^ (y >> np.uint32(1)) ^ ((np.uint32(0) - (y & np.uint32(1))) & MATRIX_A)


def next_block(a):
    """mt19937_gen: the next 624 words from the current key a."""
    b = np.empty(N, dtype=np.uint32)
    b[:N - M] = _twist(a[:N - M], a[1:N - M + 1], a[M:])
    b[N - M:2 * (N - M)] = _twist(a[N - M:2 * (N - M)], a[N - M + 1:2 * (N - M) + 1], b[:N - M])
    i = np.arange(2 * (N - M), N)
    nxt = np.where(i == N - 1, b[0], a[np.minimum(i + 1, N - 1)])
    b[2 * (N - M):] = _twist(a[2 * (N - M):], nxt, b[i - (N - M)])
    return b


def stream(key, nblk):
    """X: the key followed by nblk generated blocks."""
    out = [np.asarray(key, dtype=np.uint32)]
    for _ in range(nblk):
        out.append(next_block(out[-1]))
    return np.concatenate(out)


def temper(y):
    y = np.asarray(y, dtype=np.uint32)
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def legacy_double(w0, w1):
    a = (w0 >> np.uint32(5)).astype(np.int64).astype(np.float64)
    b = (w1 >> np.uint32(6)).astype(np.int64).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0


def draw(state, n_pre, g, log=libm_log):
    """n_pre random_sample doubles, then g standard normals, from an
    np.random.get_state() tuple -> (doubles, normals, new state tuple)."""
    _, key, pos, has_gauss, gauss = state[:5]
    key = np.asarray(key, dtype=np.uint32)
    h = 1 if (has_gauss and g > 0) else 0
    m = g - h if g > 0 else 0
    P = (m + 1) // 2
    pw = 2 * n_pre
    # enough words: grow the candidate window until P pairs are accepted
    ncand = max(16, int(P / 0.785398) + 64)
    while True:
        words = pos + pw + 4 * ncand
        X = stream(key, words // N + 2)
        T = temper(X[pos:pos + pw + 4 * ncand])
        pre = legacy_double(T[0:pw:2], T[1:pw:2])
        c = T[pw:].reshape(ncand, 4)
        x1 = 2.0 * legacy_double(c[:, 0], c[:, 1]) - 1.0
        x2 = 2.0 * legacy_double(c[:, 2], c[:, 3]) - 1.0
        r2 = x1 * x1 + x2 * x2
        acc = ~((r2 >= 1.0) | (r2 == 0.0))
        if P == 0 or acc.sum() >= P:
            break
        ncand *= 2
    normals = np.empty(g)
    new_has, new_gauss = (has_gauss, gauss) if g == 0 else (0, 0.0)
    j_end = pw
    if h:
        normals[0] = gauss
    if P > 0:
        sel = np.flatnonzero(acc)[:P]
        f = np.sqrt(-2.0 * log(r2[sel]) / r2[sel])
        pair = np.empty(2 * P)
        pair[0::2] = f * x2[sel]
        pair[1::2] = f * x1[sel]
        normals[h:] = pair[:m]
        if m & 1:
            new_has, new_gauss = 1, pair[-1]
        j_end = pw + 4 * (int(sel[-1]) + 1)
    e = pos + j_end
    if e > 0 and e % N == 0:
        blk, npos = e // N - 1, N
    else:
        blk, npos = e // N, e % N
    new_key = X[blk * N:(blk + 1) * N].copy()
    return pre, normals, ("MT19937", new_key, int(npos), int(new_has), float(new_gauss))
