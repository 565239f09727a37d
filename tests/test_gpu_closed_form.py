"""The closed-form log-sum likelihood's two evaluations on the device (DESIGN
4.3): the fp64 expansion about the step's reference pose and the double-double
form it falls back to (SLAM_PF_EXPAND_VMAX=0 forces the latter).  Bars:

  * particles clustered around the reference pose (the expansion is taken):
    weights within one ulp of the residual sum F of the double-double form
    (its own error is |dL| <= 1e-14, then both round F once) and not all
    bit-identical to it (the fast form ran);
  * particles metres away from it (the bound sends every one to the fallback):
    bit-identical to the double-double form;
  * both against the reference's factor-by-factor product (the oracle):
    identical zero sets, <= 1e-12 relative.
"""
import os

import numpy as np
import pytest

from conftest import weights_match

import pf_oracle as po

pytestmark = pytest.mark.gpu

X0 = np.array([10.0, 0.0, np.pi / 2])


def _update(px, pw, lm, z, vmax):
    from slamhip.pf import DeviceParticleFilter
    old = os.environ.get("SLAM_PF_EXPAND_VMAX")
    os.environ["SLAM_PF_EXPAND_VMAX"] = vmax
    try:
        with DeviceParticleFilter(px.shape[1], lm, likelihood="logsum", x0=tuple(X0)) as d:
            d.set_state(px[0], px[1], px[2], pw)
            out = d.update(z)
            w = d.get_state()[3]
    finally:
        if old is None:
            os.environ.pop("SLAM_PF_EXPAND_VMAX")
        else:
            os.environ["SLAM_PF_EXPAND_VMAX"] = old
    return out, w


def _world(rs, nl, n, spread, offset):
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm)
    from mylib import transform as tf
    z = tf.world2robot(X0.reshape(3, 1), lm) + rs.multivariate_normal([0, 0], p.r, nl)
    px = X0.reshape(3, 1) + offset + spread * rs.randn(3, n)
    pw = np.full(n, 1.0 / n)
    return p, lm, z, px, pw


def _residual_sums(px, lm, z):
    # sum_j |R(l_j - p) - z_j|^2 per particle (host cos / sin: only for the bar)
    c, s = np.cos(np.pi / 2 - px[2]), np.sin(np.pi / 2 - px[2])
    dx = lm[:, 0][None, :] - px[0][:, None]
    dy = lm[:, 1][None, :] - px[1][:, None]
    rx = c[:, None] * dx - s[:, None] * dy - z[:, 0][None, :]
    ry = s[:, None] * dx + c[:, None] * dy - z[:, 1][None, :]
    return (rx * rx + ry * ry).sum(axis=1)


def _oracle_weights(p, px, pw, lm, z):
    w, _ = po.likelihood_loop(px[0], px[1], px[2], pw, lm, z, p.r)
    return w


@pytest.mark.parametrize("nl,n,spread", [(100, 20000, 1e-4), (20, 5000, 2e-3), (100, 4096, 0.02)])
def test_expansion_matches_double_double_near_reference(nl, n, spread):
    rs = np.random.RandomState(nl + n)
    p, lm, z, px, pw = _world(rs, nl, n, spread, 0.0)
    out_f, wf = _update(px, pw, lm, z, "1")
    out_d, wd = _update(px, pw, lm, z, "0")
    nz = wd > 0
    assert np.array_equal(wf > 0, nz)
    rel = np.max(np.abs(wf[nz] - wd[nz]) / wd[nz])
    # both forms round the exact sum F once (the fast one after its <= 1e-14
    # error in L): they may differ by one ulp of F, i.e. 2^-53 F / sx2 in L,
    # and the two normalisations by as much again
    fmax = _residual_sums(px, lm, z).max()
    bar = 3e-14 + 2.0 ** -52 * fmax / p.r[0, 0]
    print(f"nl={nl} n={n} spread={spread}: fast vs double-double max rel {rel:.3g} (bar {bar:.3g})")
    assert rel <= bar
    assert not np.array_equal(wf, wd)
    assert out_f["max_idx"] == out_d["max_idx"]
    ref = _oracle_weights(p, px, pw, lm, z)
    weights_match(wf, ref, rtol=1e-12)


def test_far_particles_fall_back_bit_identical():
    rs = np.random.RandomState(3)
    p, lm, z, px, pw = _world(rs, 30, 3000, 0.2, np.array([[3.0], [-2.0], [0.3]]))
    _, wf = _update(px, pw, lm, z, "1")
    _, wd = _update(px, pw, lm, z, "0")
    assert np.array_equal(wf, wd)
    ref = _oracle_weights(p, px, pw, lm, z)
    weights_match(wf, ref, rtol=1e-12)
