"""CPU check of the algebra behind the closed-form log-sum likelihood
(pf_kernels.inl closed_prep_constants / likelihood_lanes): in exact
rational arithmetic,

  * the eight landmark / observation sums reproduce sum_j |R(c,s)(l_j - p) - z_j|^2
    for any particle (x, y, c, s) -- the double-double form;
  * the constants of the expansion about a reference pose (p^, c^, s^) built
    from those sums reproduce the same sum through the per-particle polynomial
    F^ + 2 (dc A + ds B) - 2 S_r.R d + (dc^2 + ds^2) L2 - 2 (dR L1).R d + NL |R d|^2
    -- the fp64 fast form;
  * V = 2 (|gx u| + |gy v| + |Srx u| + |Sry v|) + t5 bounds the magnitudes the
    kernel's fp64 part rounds (its rounding bound is 11 u V; the rotation terms
    are formed in double-double, dc and ds with their TwoSum errors);
  * the kernel's own fp64 operation order stays within u |F| + 11 u V of the
    exact sum for a bench-like cloud, and such a cloud passes the fast-form
    test V / sx2 <= 480.

No GPU: this pins the identities the kernel evaluates, independent of rounding.
"""
from fractions import Fraction as Fr

import numpy as np


def _rot(c, s, v):
    return (c * v[0] - s * v[1], s * v[0] + c * v[1])


def _direct(lm, z, x, y, c, s):
    tot = Fr(0)
    for (lx, ly), (zx, zy) in zip(lm, z):
        rx, ry = _rot(c, s, (lx - x, ly - y))
        tot += (rx - zx) ** 2 + (ry - zy) ** 2
    return tot


def _sums(lm, z):
    S = dict(ll=Fr(0), lx=Fr(0), ly=Fr(0), zz=Fr(0), zx=Fr(0), zy=Fr(0), D=Fr(0), E=Fr(0))
    for (lx, ly), (zx, zy) in zip(lm, z):
        S["ll"] += lx * lx + ly * ly
        S["lx"] += lx
        S["ly"] += ly
        S["zz"] += zx * zx + zy * zy
        S["zx"] += zx
        S["zy"] += zy
        S["D"] += zx * lx + zy * ly
        S["E"] += zy * lx - zx * ly
    return S


def _dd_form(S, nl, x, y, c, s):
    # likelihood_lanes' double-double form
    p1 = S["ll"] - 2 * (x * S["lx"] + y * S["ly"]) + nl * (x * x + y * y)
    kk = c * c + s * s
    q1 = S["D"] - (S["zx"] * x + S["zy"] * y)
    q2 = S["E"] - (S["zy"] * x - S["zx"] * y)
    return kk * p1 - 2 * (q1 * c + q2 * s) + S["zz"]


def _constants(S, nl, px, py, ch, sh):
    # closed_prep_constants
    L1x, L1y = S["lx"] - nl * px, S["ly"] - nl * py
    L2 = S["ll"] - 2 * (S["lx"] * px + S["ly"] * py) + nl * (px * px + py * py)
    Dh = S["D"] - (S["zx"] * px + S["zy"] * py)
    Eh = S["E"] - (S["zy"] * px - S["zx"] * py)
    A, B = ch * L2 - Dh, sh * L2 - Eh
    Srx = ch * L1x - sh * L1y - S["zx"]
    Sry = sh * L1x + ch * L1y - S["zy"]
    F = (ch * ch + sh * sh) * L2 - 2 * (Dh * ch + Eh * sh) + S["zz"]
    return dict(F=F, A=A, B=B, Srx=Srx, Sry=Sry, L2=L2, L1x=L1x, L1y=L1y, NL=Fr(nl))


def _expansion(K, px, py, ch, sh, x, y, c, s):
    # likelihood_lanes' fast form, term by term (exact)
    dx, dy, dc, ds = x - px, y - py, c - ch, s - sh
    u, v = _rot(c, s, (dx, dy))
    t1 = dc * K["A"] + ds * K["B"]
    t2 = K["Srx"] * u + K["Sry"] * v
    gx, gy = dc * K["L1x"] - ds * K["L1y"], ds * K["L1x"] + dc * K["L1y"]
    t4 = gx * u + gy * v
    t3 = (dc * dc + ds * ds) * K["L2"]
    t5 = (u * u + v * v) * K["NL"]
    F = K["F"] + 2 * t1 - 2 * t2 + t3 - 2 * t4 + t5
    # magnitudes the fp64 part rounds: the translation terms (the rotation
    # terms are formed in double-double)
    mags = (2 * abs(K["Srx"] * u) + 2 * abs(K["Sry"] * v) + 2 * abs(gx * u) + 2 * abs(gy * v)
            + abs(t5))
    V = 2 * (abs(u) * (abs(gx) + abs(K["Srx"])) + abs(v) * (abs(gy) + abs(K["Sry"]))) + t5
    return F, mags, V


def _fr(v):
    return Fr(float(v))


def test_closed_form_identities_exact():
    rs = np.random.RandomState(11)
    for trial in range(12):
        nl = int(rs.randint(1, 9))
        lm = [(_fr(a), _fr(b)) for a, b in rs.uniform(-10, 10, (nl, 2))]
        pose = rs.uniform(-5, 5, 3)
        z = [(_fr(a), _fr(b)) for a, b in rs.uniform(-12, 12, (nl, 2))]
        S = _sums(lm, z)
        # reference pose: doubles, (c^, s^) need not be a unit vector
        px, py = _fr(pose[0]), _fr(pose[1])
        ch, sh = _fr(np.cos(np.pi / 2 - pose[2])), _fr(np.sin(np.pi / 2 - pose[2]))
        K = _constants(S, nl, px, py, ch, sh)
        assert K["F"] == _direct(lm, z, px, py, ch, sh)
        for _ in range(6):
            sc = 10.0 ** rs.uniform(-6, 0.5)
            x, y = _fr(pose[0] + sc * rs.randn()), _fr(pose[1] + sc * rs.randn())
            th = pose[2] + sc * rs.randn()
            c, s = _fr(np.cos(np.pi / 2 - th)), _fr(np.sin(np.pi / 2 - th))
            ref = _direct(lm, z, x, y, c, s)
            assert _dd_form(S, nl, x, y, c, s) == ref
            F, mags, V = _expansion(K, px, py, ch, sh, x, y, c, s)
            assert F == ref
            assert V >= mags


def _fma(a, b, c):
    return float(Fr(a) * Fr(b) + Fr(c))


def _two_sum(h, b):
    t = h + b
    bb = t - h
    return t, (h - (t - bb)) + (b - bb)


def _kernel_fast_form(Kd, K, x, y, c, s, nl):
    """likelihood_lanes' fast form in its fp64 operation order (fma = exact
    product + one rounding): returns (F, V)."""
    dx, dy = x - Kd["px"], y - Kd["py"]
    dc, ds = c - Kd["ch"], s - Kd["sh"]
    dcb, dsb = dc - c, ds - s
    dce = (c - (dc - dcb)) + (-Kd["ch"] - dcb)
    dse = (s - (ds - dsb)) + (-Kd["sh"] - dsb)
    Ah, Al = K["Ah"], K["Al"]
    Bh, Bl = K["Bh"], K["Bl"]
    L2h, L2l = K["L2h"], K["L2l"]
    p1 = dc * Ah
    e1 = _fma(dc, Ah, -p1)
    p2 = ds * Bh
    e2 = _fma(ds, Bh, -p2)
    q1 = dc * dc
    f1 = _fma(dc, dc, -q1)
    q2 = ds * ds
    f2 = _fma(ds, ds, -q2)
    a2 = q1 + q2
    a2b = a2 - q1
    a2e = ((q1 - (a2 - a2b)) + (q2 - a2b)) + (f1 + f2)
    p3 = a2 * L2h
    a2x = a2e + 2.0 * _fma(dce, dc, dse * ds)
    e3 = _fma(a2, L2h, -p3) + _fma(a2x, L2h, a2 * L2l)
    u = _fma(c, dx, -(s * dy))
    v = _fma(s, dx, c * dy)
    t2 = _fma(Kd["Srx"], u, Kd["Sry"] * v)
    gx, gy = _fma(dc, Kd["L1x"], -(ds * Kd["L1y"])), _fma(ds, Kd["L1x"], dc * Kd["L1y"])
    t4 = _fma(gx, u, gy * v)
    t5 = _fma(u, u, v * v) * nl
    h, lo = _two_sum(K["Fh"], 2.0 * p1)
    h, l2 = _two_sum(h, 2.0 * p2)
    lo += l2
    h, l3 = _two_sum(h, p3)
    lo += l3
    rot_lo = _fma(2.0, (e1 + e2) + (_fma(dc, Al, ds * Bl) + _fma(dce, Ah, dse * Bh)), e3)
    lo = lo + ((K["Fl"] + rot_lo) + _fma(-2.0, t2 + t4, t5))
    F = h + lo
    V = _fma(2.0, _fma(abs(u), abs(gx) + abs(Kd["Srx"]), abs(v) * (abs(gy) + abs(Kd["Sry"]))), t5)
    return F, V


def _split(q):
    h = float(q)
    return h, float(q - Fr(h))


def test_expansion_rounding_within_bound_for_a_cloud():
    """The kernel's fp64 evaluation of the expansion, for a cloud with the
    bench's per-step spread around the reference pose (velocity model,
    a1..a6 = 0.1 at v = 1.75 m/s: ~1 cm, ~0.013 rad), stays within
    u |F| + 11 u V of the exact sum, and V sx2^-1 <= 480 (the kernel's
    fast-form test) for the cloud."""
    rs = np.random.RandomState(5)
    nl = 100
    lm_f = rs.uniform(-10, 10, (nl, 2))
    pose = np.array([10.0, 0.0, np.pi / 2])
    c0, s0 = np.cos(np.pi / 2 - pose[2]), np.sin(np.pi / 2 - pose[2])
    rel = lm_f - pose[:2]
    zf = np.column_stack([c0 * rel[:, 0] - s0 * rel[:, 1], s0 * rel[:, 0] + c0 * rel[:, 1]])
    zf += 0.3 * rs.randn(nl, 2)
    lm = [tuple(map(_fr, r)) for r in lm_f]
    z = [tuple(map(_fr, r)) for r in zf]
    S = _sums(lm, z)
    K = _constants(S, nl, _fr(pose[0]), _fr(pose[1]), _fr(c0), _fr(s0))
    Kd = {k: float(v) for k, v in K.items()}
    Kd.update(px=pose[0], py=pose[1], ch=c0, sh=s0)
    Kx = {}
    for name, key in (("F", "F"), ("A", "A"), ("B", "B"), ("L2", "L2")):
        Kx[name + "h"], Kx[name + "l"] = _split(K[key])
    u53 = 2.0 ** -53
    vs = []
    for _ in range(40):
        x, y = pose[0] + 0.017 * rs.randn(), pose[1] + 0.017 * rs.randn()
        th = pose[2] + 0.022 * rs.randn()
        c, s = np.cos(np.pi / 2 - th), np.sin(np.pi / 2 - th)
        F, V = _kernel_fast_form(Kd, Kx, x, y, c, s, nl)
        exact = _direct(lm, z, _fr(x), _fr(y), _fr(c), _fr(s))
        assert abs(Fr(F) - exact) <= Fr(u53) * abs(exact) + Fr(11 * u53) * Fr(V)
        vs.append(V / 0.09)
    assert max(vs) <= 480.0, max(vs)
