"""CPU checks of the device RNG's two restatements (no GPU):

* oracle/mt_oracle.py: NumPy's legacy stream in the device pipeline's form
  (generated-ahead key sequence, four-word candidates, first P accepted pairs,
  the state NumPy leaves) against np.random.RandomState itself -- bit-exact
  draws and identical get_state() tuples;
* glibc's log as the device evaluates it (libslam_hip's host copy of
  mt19937.hpp's glibc_log, table read from this process's libm) against the C
  library's log() -- bit-exact.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

import mt_oracle as mo


def _same_state(a, b):
    assert a[0] == b[0]
    np.testing.assert_array_equal(np.asarray(a[1], np.uint32), np.asarray(b[1], np.uint32))
    assert (int(a[2]), int(a[3])) == (int(b[2]), int(b[3]))
    assert np.float64(a[4]).view(np.uint64) == np.float64(b[4]).view(np.uint64)


@pytest.mark.parametrize("seed,warm,g", [(0, 0, 1), (1, 3, 2), (2, 1, 3), (3, 0, 1000),
                                         (4, 311, 1501), (5, 312, 6000)])
def test_oracle_standard_normal_matches_numpy(seed, warm, g):
    rs = np.random.RandomState(seed)
    rs.random_sample(warm)                       # misalign pos (312 doubles: pos = 624)
    _, out, st = mo.draw(rs.get_state(), 0, g)
    ref = rs.standard_normal(g)
    np.testing.assert_array_equal(out.view(np.uint64), ref.view(np.uint64))
    _same_state(st, rs.get_state())


def test_oracle_interleaved_calls_match_numpy():
    """rand() between normal draws leaves the cached normal alone (the PF's
    resample offset, particle_filter.py:214, between mvn draws)."""
    rs = np.random.RandomState(17)
    st = rs.get_state()
    for n_pre, g in [(1, 5), (3, 1), (0, 2), (1, 7), (2, 0), (0, 1), (1, 4)]:
        pre, out, st = mo.draw(st, n_pre, g)
        np.testing.assert_array_equal(pre, rs.random_sample(n_pre))
        np.testing.assert_array_equal(out.view(np.uint64), rs.standard_normal(g).view(np.uint64))
        _same_state(st, rs.get_state())


def test_glibc_log_restatement_bit_exact():
    from slamhip import rng
    libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
    libm.log.restype = ctypes.c_double
    libm.log.argtypes = [ctypes.c_double]
    rs = np.random.RandomState(0)
    x = np.concatenate([rs.random_sample(60000),                       # polar r2 range
                        1.0 - rs.random_sample(30000) * 2.0 ** -4,     # |x - 1| < 2^-4 branch
                        1.0 + rs.random_sample(10000) * 0.0645,
                        np.ldexp(0.5 + rs.random_sample(20000), rs.randint(-1070, 1000, 20000)),
                        [2.0 ** -1074, 2.0 ** -1060, 1e-310, 1.0, 2.0, 0.5]])
    x = x[x > 0]
    got = rng.glibc_log(x)
    ref = np.array([libm.log(float(v)) for v in x])
    bad = np.flatnonzero(got.view(np.uint64) != ref.view(np.uint64))
    assert bad.size == 0, (x[bad[:5]], got[bad[:5]], ref[bad[:5]])


@pytest.mark.parametrize("n_words", [1, 623, 624, 20000, 3 * 624 * 1000 + 17])
def test_jump_ahead_window(n_words):
    """Jump-ahead (x^n mod MT19937's characteristic polynomial, applied as an
    XOR of shifted windows) lands on the window the recurrence reaches."""
    from slamhip import rng
    key = np.asarray(np.random.RandomState(n_words).get_state()[1], np.uint32)
    start = 5                                   # a window inside the generated stream
    X = mo.stream(key, (start + n_words + 624) // 624 + 2)
    win = X[start:start + 624]
    got = rng.jump_window(win, n_words)
    ref = X[start + n_words:start + n_words + 624]
    np.testing.assert_array_equal(got[1:], ref[1:])
    assert (got[0] ^ ref[0]) >> 31 == 0
