"""The device-RNG tables in csrc/fastmath.hpp equal tools/gen_rng_tables.py's
mpmath output bit for bit (sin/cos(2 pi j/256) and the log slots' invc and
-log(invc) correctly rounded)."""
import pathlib
import re
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
mp = pytest.importorskip("mpmath")
sys.path.insert(0, str(ROOT / "tools"))
import gen_rng_tables as gen  # noqa: E402

HEX = r"-?0x[0-9a-fA-F.]+p[-+]?\d+"


def _table(name):
    src = (ROOT / "slam-robot_simu_amd/csrc/fastmath.hpp").read_text()
    m = re.search(name + r"\[256\] = \{(.*?)\n\};", src, re.S)
    assert m, name
    return [float.fromhex(x) for x in re.findall(HEX, m.group(1))]


def _flat(pairs):
    return [v for p in pairs for v in p]


def test_sincos_table():
    assert _table("kRngSinCos256") == _flat(gen.sincos_table())


def test_log_tables():
    li, ll = gen.log_tables()
    assert _table("kRngLogInvHi") == _flat(li)
    assert _table("kRngLogLo") == ll
    # exactly 1 beside m = 1, so r = m - 1 is exact there
    assert li[127][0] == 1.0 and li[128][0] == 1.0
