"""heading_sincos_tab (csrc/fastmath.hpp): the velocity model's sin/cos of a
wrapped heading (motion_model.py:50-56) from the device RNG's LDS table of
(sin, cos)(2 pi j / 256), restated here operation by operation (every fma
exact by rational arithmetic, every other operation an IEEE double) and held
against mpmath: within 2 ulp of sin / cos over the heading range the kernel
sends it, |x| <= pi + 0.1 (the ulp of the larger of the value and 2^-20:
beside the zeros at multiples of pi/2 the two-part reduction leaves an
absolute ~2e-31, e.g. 7 ulp of sin(fl(pi)) = 1.2e-16, against a physical
effect of that absolute size times the turn radius).  fast_sincos (the
fdlibm kernels, three-part reduction) is < 1 ulp; the
predict's parity bars (tests/test_gpu_c2.py: 1e-12 (|ref| + |v/w|)) sit
four orders above either."""
import math
import pathlib
import re
from fractions import Fraction

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
mp = pytest.importorskip("mpmath")
HEX = r"-?0x[0-9a-fA-F.]+p[-+]?\d+"


def _table():
    src = (ROOT / "slam-robot_simu_amd/csrc/fastmath.hpp").read_text()
    m = re.search(r"kRngSinCos256\[256\] = \{(.*?)\n\};", src, re.S)
    v = [float.fromhex(x) for x in re.findall(HEX, m.group(1))]
    return [(v[2 * k], v[2 * k + 1]) for k in range(256)]


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def heading_sincos_tab(x, T):
    k128pi = 40.74366543152521
    hi, lo = float.fromhex("0x1.921fb54442dp-6"), float.fromhex("0x1.8469898cc5170p-54")
    j = float(np.rint(x * k128pi))
    r = fma(-j, lo, fma(-j, hi, x))
    ts, tc = T[int(j) & 255]
    z = r * r
    sr = fma(r * z, fma(z, fma(z, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), r)
    cr = fma(z, fma(z, fma(z, -1.0 / 720.0, 1.0 / 24.0), -0.5), 1.0)
    return fma(ts, cr, tc * sr), fma(tc, cr, -(ts * sr))


def test_constants_split_pi_over_128():
    mp.mp.prec = 200
    hi, lo = float.fromhex("0x1.921fb54442dp-6"), float.fromhex("0x1.8469898cc5170p-54")
    assert abs(mp.mpf(hi) + mp.mpf(lo) - mp.pi / 128) < mp.mpf(2) ** -105
    assert (hi * 2 ** 50).is_integer()                   # 45 significant bits: j hi exact, |j| <= 130


def test_heading_sincos_within_2ulp():
    T = _table()
    rs = np.random.RandomState(3)
    xs = list(rs.uniform(-math.pi - 0.1, math.pi + 0.1, 3000))
    xs += [0.0, -0.0, math.pi, -math.pi, math.pi / 2, -math.pi / 2, math.pi / 256, 3 * math.pi / 256,
           math.pi / 128, 1e-300, 5e-324, -1e-17]
    xs += [k * math.pi / 128 + d for k in range(-128, 129, 7) for d in (-1e-12, 0.0, 1e-12)]
    mp.mp.prec = 120
    worst = 0.0
    for x in xs:
        s, c = heading_sincos_tab(x, T)
        for got, ref in ((s, mp.sin(mp.mpf(x))), (c, mp.cos(mp.mpf(x)))):
            ulp = math.ulp(max(abs(float(ref)), 2.0 ** -20))
            err = float(abs(mp.mpf(got) - ref)) / ulp
            worst = max(worst, err)
    print("heading_sincos_tab worst error:", worst, "ulp")
    assert worst <= 2.0
