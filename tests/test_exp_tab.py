"""Host restatement of fastmath.hpp's exp_tab (the product likelihood's exp):
the header's 64-entry table, k = round(x 64/ln2) by the 1.5 2^52 shift,
Cody-Waite reduction, degree-5 polynomial, every fma emulated exactly
(Fraction arithmetic, one rounding).  Pins the header's accuracy claim:
under 0.9 ulp against mpmath's correctly rounded exp on arguments the
likelihood produces (x = -q/2 <= 0, normal results)."""
import math
import pathlib
import random
import re
from fractions import Fraction

import pytest

mp = pytest.importorskip("mpmath")
ROOT = pathlib.Path(__file__).resolve().parents[1]
HEX = r"-?0x[0-9a-fA-F.]+p[-+]?\d+"


def _table():
    src = (ROOT / "slam-robot_simu_amd/csrc/fastmath.hpp").read_text()
    m = re.search(r"kExpTab64\[64\] = \{(.*?)\n\};", src, re.S)
    v = [float.fromhex(x) for x in re.findall(HEX, m.group(1))]
    return list(zip(v[0::2], v[1::2]))


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def exp_tab(x, tab):
    k_inv = float.fromhex("0x1.71547652b82fep+6")
    neg_hi = float.fromhex("-0x1.62e42ff000000p-7")
    neg_lo = float.fromhex("0x1.718432a1b0e26p-41")
    shift = float.fromhex("0x1.8p52")
    kdm = fma(x, k_inv, shift)
    kd = kdm - shift
    r = fma(kd, neg_lo, fma(kd, neg_hi, x))
    ki = int(kd)                       # the device reads it from kdm's low word
    tx, ty = tab[ki & 63]
    r2 = r * r
    c45 = fma(r, 1.0 / 120.0, 1.0 / 24.0)
    c23 = fma(r, 1.0 / 6.0, 0.5)
    p = fma(r2, fma(r2, c45, c23), r)
    v = tx + fma(tx, p, ty)
    return 0.0 if x < -746.0 else math.ldexp(v, ki >> 6)


def test_exp_tab_under_0p9_ulp():
    tab = _table()
    mp.mp.dps = 40
    rng = random.Random(7)
    xs = [-rng.uniform(0.0, 700.0) for _ in range(1500)] + [-rng.uniform(0.0, 1e-3) for _ in range(200)]
    worst = 0.0
    for x in xs:
        got = exp_tab(x, tab)
        ref = mp.exp(mp.mpf(x))
        ulp = math.ulp(float(ref))
        worst = max(worst, abs(float((mp.mpf(got) - ref) / ulp)))
    assert worst < 0.9, worst


def exp_nhalf(y, tab):
    """fastmath.hpp exp_nhalf: exp(-y/2) on doubled intermediates, table t.x halved."""
    k_inv = float.fromhex("0x1.71547652b82fep+6")
    neg_hi = float.fromhex("-0x1.62e42ff000000p-7")
    neg_lo = float.fromhex("0x1.718432a1b0e26p-41")
    shift = float.fromhex("0x1.8p52")
    kdm = fma(y, -0.5 * k_inv, shift)
    kd = kdm - shift
    r = fma(kd, 2.0 * neg_lo, fma(kd, 2.0 * neg_hi, -y))
    ki = int(kd)
    tx, ty = tab[ki & 63]
    tx = tx * 0.5
    r2 = r * r
    c45 = fma(r, (1.0 / 120.0) / 16.0, (1.0 / 24.0) / 8.0)
    c23 = fma(r, (1.0 / 6.0) / 4.0, 0.25)
    p = fma(r2, fma(r2, c45, c23), r)
    v = fma(tx, 2.0, fma(tx, p, ty))
    return 0.0 if y > 1492.0 else math.ldexp(v, ki >> 6)


def test_exp_nhalf_bits_equal_exp_tab():
    """The product factor's exp(-q/2) without forming q/2 gives exp_tab(-q/2)'s bits
    (q >= 0 in the likelihood; also the rho path's 2|a|, tiny and subnormal q, the range edges)."""
    tab = _table()
    rng = random.Random(11)
    ys = [rng.uniform(0.0, 1500.0) for _ in range(1500)] + [rng.uniform(0.0, 1e-3) for _ in range(300)]
    ys += [math.ldexp(rng.uniform(1.0, 2.0), -rng.randrange(20, 1074)) for _ in range(300)]
    ys += [0.0, 5e-324, 2.2250738585072014e-308, 1490.0, 1491.99, 1492.0, 1492.5, 1e5]
    ys += [2.0 * rng.uniform(0.0, 700.0) for _ in range(300)]
    for y in ys:
        x = -y * 0.5
        want = exp_tab(x, tab)
        got = exp_nhalf(y, tab)
        assert got == want and math.copysign(1.0, got) == math.copysign(1.0, want), (y, got, want)
