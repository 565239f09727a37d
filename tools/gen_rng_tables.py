"""Generate the device-RNG tables of csrc/fastmath.hpp (kRngSinCos256,
kRngLogInvHi, kRngLogLo) with mpmath at 60 digits, or check the header's
copies against them (tests/test_rng_tables.py).

    python tools/gen_rng_tables.py            # print the three tables as C++

Slots (fastmath.hpp rng_log_tab): j = top 7 fraction bits of m | (m >= 1) << 7,
m in [sqrt(1/2), sqrt(2)); c = the slot's midpoint, invc = 1 / c rounded to
2^-10 (exactly 1 in slots 127 and 128, beside m = 1), -log(invc) split hi + lo.
"""
import mpmath as mp

mp.mp.dps = 60


def _d(x):
    return float(mp.mpf(x))            # nearest double (mpf -> float rounds to nearest)


def sincos_table():
    out = []
    for j in range(256):
        a = 2 * mp.pi * j / 256
        s, c = mp.sin(a), mp.cos(a)
        # exact zeros at the quarter turns (mpmath leaves ~1e-61 there)
        out.append((0.0 if j % 128 == 0 else _d(s), 0.0 if j % 128 == 64 else _d(c)))
    return out


def log_tables():
    li, ll = [], []
    for j in range(256):
        f7, top = j & 0x7F, j >> 7
        lo = (1 + mp.mpf(f7) / 128) * (1 if top else mp.mpf(1) / 2)
        c = lo + (mp.mpf(1) / 256 if top else mp.mpf(1) / 512)
        invc = mp.mpf(1) if j in (127, 128) else mp.nint(mp.mpf(1024) / c) / 1024
        v = -mp.log(invc)
        hi = _d(v)
        li.append((float(invc), hi))
        ll.append(_d(v - mp.mpf(hi)))
    return li, ll


def _fmt(x):
    return float.hex(x) if x != 0 else "0x0.0p+0"


def main():
    sc = sincos_table()
    li, ll = log_tables()
    print("__device__ __constant__ const double2 kRngSinCos256[256] = {")
    for s, c in sc:
        print(f"    {{{_fmt(s)}, {_fmt(c)}}},")
    print("};")
    print("__device__ __constant__ const double2 kRngLogInvHi[256] = {")
    for a, b in li:
        print(f"    {{{_fmt(a)}, {_fmt(b)}}},")
    print("};")
    print("__device__ __constant__ const double kRngLogLo[256] = {")
    for x in ll:
        print(f"    {_fmt(x)},")
    print("};")


if __name__ == "__main__":
    main()
