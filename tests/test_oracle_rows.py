"""CPU checks of the oracle's O(n m) EKF-SLAM row form against its dense
restatement (the C4 GPU test compares the device with the row form), and of
the velocity-model EKF restatement (N1)."""
import numpy as np
import pytest

from conftest import golden

import ekf_oracle as eo
import pf_oracle as po


def test_update_rows_matches_dense_step():
    rs = np.random.RandomState(0)
    n_lm, k, dt = 60, 7, 0.1
    n = 3 + 3 * n_lm
    lm = np.column_stack([rs.uniform(-20, 20, (n_lm, 2)), rs.uniform(-np.pi, np.pi, n_lm)])
    mu = np.concatenate([[1.0, -2.0, 0.4], (lm + rs.normal(0, 0.3, lm.shape)).ravel()])
    A = rs.normal(0, 0.05, (n, 12))
    P = A @ A.T + np.diag(rs.uniform(0.01, 0.2, n))
    q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
    noise = (0.05, np.deg2rad(2.0), np.deg2rad(2.0))
    ids = rs.choice(n_lm, k, replace=False)
    ctl = (1.5, 0.2)
    xr = eo.ekf_motion(mu[:3], dt, *ctl)
    obs = np.array([eo.scan_predict(xr, lm[j]) for j in ids]) + rs.normal(0, 0.01, (k, 3))
    mu_d, P_d = eo.ekfslam_step(mu, P, ctl, ids, obs, dt, q, noise)
    # the same step: dense predict, then the row form of the update
    F = eo.ekf_jacobian(mu[:3], dt, ctl[0])
    mu_p = mu.copy()
    mu_p[:3] = xr
    Pp = P.copy()
    Pp[:3, :] = F @ Pp[:3, :]
    Pp[:, :3] = Pp[:, :3] @ F.T
    Pp[:3, :3] += q
    idx = np.concatenate([[0, 1, 2], (3 + 3 * ids[:, None] + np.arange(3)).ravel()])
    rows = np.sort(rs.choice(n, 40, replace=False))
    mu_r, P_r = eo.ekfslam_update_rows(mu_p, Pp[idx], Pp[rows], rows, ids, obs, noise)
    np.testing.assert_allclose(mu_r, mu_d, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(P_r, P_d[rows], rtol=0, atol=1e-12 * np.abs(P_d).max())


# ------------------------------------------------------------------ N1
# EKF driven by motion_model.py (north_star): f = moveWithoutNoise pinned to
# the reference's outputs (motion.npz), its Jacobians by central differences,
# and the process noise V M V^T (+ gamma) against the sample covariance of the
# reference's own noisy model (pf_oracle.motion_velocity, pinned to motion.npz).


@pytest.mark.parametrize("c", range(3))
def test_velocity_ekf_motion_is_move_without_noise(c):
    g = golden("motion")
    dt, *alphas, v, w = g[f"case{c}"]
    out = np.array([eo.velocity_motion(p, v, w, dt) for p in g["poses"]])
    assert np.array_equal(out, g[f"clean{c}"])


def test_velocity_ekf_jacobians_central_differences():
    rs = np.random.RandomState(2)
    for _ in range(50):
        x = np.array([rs.uniform(-5, 5), rs.uniform(-5, 5), rs.uniform(-3, 3)])
        v, om, dt = rs.uniform(0.1, 2.0), rs.uniform(0.05, 1.5) * rs.choice([-1, 1]), 0.1
        G, V = eo.velocity_jacobians(x, v, om, dt)
        h = 1e-6
        dth = (eo.velocity_motion(x + [0, 0, h], v, om, dt) - eo.velocity_motion(x - [0, 0, h], v, om, dt)) / (2 * h)
        dv = (eo.velocity_motion(x, v + h, om, dt) - eo.velocity_motion(x, v - h, om, dt)) / (2 * h)
        dw = (eo.velocity_motion(x, v, om + h, dt) - eo.velocity_motion(x, v, om - h, dt)) / (2 * h)
        np.testing.assert_allclose(G[:2, 2], dth[:2], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(V[:, 0], dv, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(V[:, 1], dw, rtol=1e-6, atol=1e-8)


def test_velocity_process_noise_matches_sampled_motion():
    rs = np.random.RandomState(9)
    alphas = (0.06, 0.04, 0.05, 0.06, 0.05, 0.03)     # small: the linearisation regime
    v, om, dt = 1.2, 0.9, 0.5
    x = np.array([1.0, -2.0, 0.4])
    n = 400000
    g = rs.standard_normal((n, 3))
    xs, ys, ts = po.motion_velocity(np.full(n, x[0]), np.full(n, x[1]), np.full(n, x[2]), v, om, dt,
                                    alphas, g)
    emp = np.cov(np.stack([xs, ys, ts]), bias=True)
    _, Pm, _, Qv = eo.velocity_predict(x, np.zeros((3, 3)), v, om, dt, alphas)
    np.testing.assert_allclose(Pm, Qv)
    np.testing.assert_allclose(np.diag(emp), np.diag(Qv), rtol=0.02)
    np.testing.assert_allclose(emp[0, 1] / np.sqrt(emp[0, 0] * emp[1, 1]),
                               Qv[0, 1] / np.sqrt(Qv[0, 0] * Qv[1, 1]), atol=0.02)


# ------------------------------------------------- the oracle's thread pool
def test_likelihood_products_threaded_bit_identical():
    """The large lockstep runs (tests/test_gpu_run_oracle.py) form the
    reference's per-particle products over a thread pool in particle chunks;
    every row must be bit-identical to the one-batch form (incl. a ragged last
    chunk and the underflow tail)."""
    rs = np.random.RandomState(3)
    n, nl = 200_003, 37
    lm = rs.uniform(-10, 10, (nl, 2))
    x, y = rs.normal(0, 3, n), rs.normal(0, 3, n)
    th = rs.uniform(-np.pi, np.pi, n)
    z = po.to_robot_frame(np.array([0.5, -0.2, 1.0]), lm)
    r = np.diag([0.3, 0.3]) ** 2
    one = po.landmark_factors(x, y, th, lm, z, r).prod(axis=1)
    many = po.likelihood_products(x, y, th, lm, z, r, threads=4, chunk=1 << 14)
    assert np.array_equal(one, many)
    assert (one == 0).any() and (one > 0).any()
