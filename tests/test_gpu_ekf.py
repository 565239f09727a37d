"""EKF on the GPU through the C-ABI.

* The drop-in ExtendedKalmanFilter against the reference's own 360-step
  main_ekf trajectory (tests/golden/ekf.npz, pinned): host-side truth,
  dead reckoning and observations bit-exact; the filter's x_hat_m, x_hat and P
  within 1e-11 relative (ocml sin/cos vs glibc, 2x2 inverse by cofactors vs
  LAPACK getri).
* Batched filters (independent observation streams) against the oracle's
  ekf_update, one filter at a time.
* EKF-SLAM (BASELINE config 4, parity against the oracle restatement only --
  the reference has no EKF-SLAM): predict + rank-3k update with the
  covariance stored as a lower triangle and updated by fp64 MFMA tiles.
"""
import numpy as np
import pytest

import ekf_oracle as eo
from conftest import golden

pytestmark = pytest.mark.gpu


def test_dropin_main_ekf_matches_reference_fixture():
    from extended_kalman_filter import ExtendedKalmanFilter
    g = golden("ekf")
    np.random.seed(int(g["seed"]))
    ekf = ExtendedKalmanFilter(100)
    steps = len(g["P"])
    out = {k: [] for k in ["x_true", "x_dr", "z", "x_hat_m", "P", "x_hat"]}
    for _ in range(steps):
        xt, xdr, z, xm, P = ekf.main_ekf()
        out["x_true"].append(xt[:, 0])
        out["x_dr"].append(xdr[:, 0])
        out["z"].append(z[:, 0])
        out["x_hat_m"].append(xm[:, 0])
        out["P"].append(P)
        out["x_hat"].append(ekf.x_hat[:, 0])
    for k in ["x_true", "x_dr", "z"]:
        np.testing.assert_array_equal(np.array(out[k]), g[k], err_msg=k)
    for k in ["x_hat_m", "x_hat", "P"]:
        np.testing.assert_allclose(np.array(out[k]), g[k], rtol=1e-11, atol=1e-14, err_msg=k)


@pytest.mark.parametrize("batch", [1, 257, 4096])
def test_batched_run_matches_oracle(batch):
    from slamhip.ekf import DeviceEKF
    p = eo.EKFParams()
    rs = np.random.RandomState(batch)
    steps = 40
    x0 = p.x0 + rs.normal(0, 0.1, (batch, 3))
    dev = DeviceEKF(batch)
    try:
        dev.set_state(x0, np.repeat(p.p0.reshape(1, 9), batch, 0))
        # observations along the reference circle with noise
        t = np.arange(1, steps + 1) * p.dt * p.omega
        base = np.stack([10 * np.cos(t), 10 * np.sin(t)], 1)
        z_all = base[:, None, :] + rs.normal(0, 1.0, (steps, batch, 2))
        xh = dev.run(z_all)
        xs, Ps = dev.get_state()
    finally:
        dev.close()
    check = range(batch) if batch <= 257 else rs.choice(batch, 200, replace=False)
    for b in check:
        x, P = x0[b].copy(), p.p0.copy()
        for s in range(steps):
            _, x, P = eo.ekf_update(x, P, z_all[s, b], p)
            np.testing.assert_allclose(xh[s, b], x, rtol=1e-11, atol=1e-12)
        np.testing.assert_allclose(Ps[b], P, rtol=1e-10, atol=1e-15)
        np.testing.assert_allclose(xs[b], x, rtol=1e-11, atol=1e-12)


def test_step_with_control_matches_oracle():
    from extended_kalman_filter import ExtendedKalmanFilter
    p = eo.EKFParams()
    ekf = ExtendedKalmanFilter(100)
    x, P = p.x0.copy(), p.p0.copy()
    rs = np.random.RandomState(5)
    for s in range(60):
        ctl = (p.vel * (1 + 0.3 * np.sin(s)), p.omega * (1 + 0.5 * np.cos(s)))
        z = x[:2] + rs.normal(0, 1, 2)
        xh, Pg = ekf.step(ctl, z.reshape(2, 1))
        _, x, P = eo.ekf_update(x, P, z, p, control=ctl)
        np.testing.assert_allclose(xh[:, 0], x, rtol=1e-11, atol=1e-12)
        np.testing.assert_allclose(Pg, P, rtol=1e-10, atol=1e-15)


def _slam_world(n_lm, seed):
    rs = np.random.RandomState(seed)
    lm = np.column_stack([rs.uniform(-30, 30, (n_lm, 2)), rs.uniform(-np.pi, np.pi, n_lm)])
    mu = np.concatenate([[0.0, 0.0, 0.3], (lm + rs.normal(0, 0.2, lm.shape)).ravel()])
    n = mu.size
    A = rs.normal(0, 0.02, (n, n // 3 + 1))
    P = A @ A.T + np.diag(np.concatenate([[0.01, 0.01, 0.002], np.full(n - 3, 0.04)]))
    P = 0.5 * (P + P.T)
    return rs, lm, mu, P


@pytest.mark.parametrize("n_lm,k,steps", [(50, 8, 12), (300, 20, 5), (700, 40, 3)])
def test_ekfslam_matches_oracle(n_lm, k, steps):
    from slamhip.ekf import DeviceEKFSLAM
    rs, lm, mu, P = _slam_world(n_lm, n_lm)
    dt = 0.1
    q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
    noise = (0.05, np.deg2rad(2.0), np.deg2rad(2.0))
    dev = DeviceEKFSLAM(n_lm, dt=dt, q_robot=q, noise=noise)
    try:
        dev.set_state(mu, P)
        mu_g, P_g = dev.get_state()
        np.testing.assert_array_equal(mu_g, mu)
        np.testing.assert_array_equal(np.tril(P_g), np.tril(P))
        xr = mu[:3].copy()
        for s in range(steps):
            ctl = (1.0, 0.1)
            xr = eo.ekf_motion(xr, dt, *ctl)
            ids = rs.choice(n_lm, k, replace=False)
            obs = np.array([eo.scan_predict(xr, lm[j]) for j in ids])
            obs[:, 0] *= 1 + rs.normal(0, 0.01, k)
            obs[:, 1:] += rs.normal(0, 0.01, (k, 2))
            dev.step(ctl, ids, obs)
            mu, P = eo.ekfslam_step(mu, P, ctl, ids, obs, dt, q, noise)
            mu_g, P_g = dev.get_state()
            scale = np.abs(P).max()
            np.testing.assert_allclose(mu_g, mu, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(P_g, 0.5 * (P + P.T), rtol=0, atol=1e-9 * scale)
        t = dev.timing()
        assert t["rank_update_ms"] > 0
    finally:
        dev.close()


def test_ekfslam_predict_only_and_init_diag():
    from slamhip.ekf import DeviceEKFSLAM
    n_lm = 130
    rs, lm, mu, P = _slam_world(n_lm, 1)
    dev = DeviceEKFSLAM(n_lm)
    try:
        dg = np.abs(rs.normal(1, 0.1, 3 + 3 * n_lm))
        dev.init_diag(mu, dg)
        mu_g, P_g = dev.get_state()
        np.testing.assert_array_equal(P_g, np.diag(dg))
        dev.set_state(mu, P)
        ctl = (0.7, -0.2)
        dev.predict(ctl)
        mu_g, P_g = dev.get_state()
        # oracle prediction (the update part of ekfslam_step skipped)
        F = eo.ekf_jacobian(mu[:3], 0.1, ctl[0])
        mu_o = mu.copy()
        mu_o[:3] = eo.ekf_motion(mu[:3], 0.1, *ctl)
        P_o = P.copy()
        P_o[:3, :] = F @ P_o[:3, :]
        P_o[:, :3] = P_o[:, :3] @ F.T
        P_o[:3, :3] += np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
        np.testing.assert_allclose(mu_g, mu_o, rtol=1e-14, atol=1e-15)
        np.testing.assert_allclose(P_g, 0.5 * (P_o + P_o.T), rtol=1e-13, atol=1e-16)
    finally:
        dev.close()
