"""N1: the EKF step driven by motion_model.py (north_star: "the
extended_kalman_filter.py Jacobian + covariance-update step driven by
motion_model.py") on the GPU, against the oracle's restatement
(ekf_oracle.velocity_predict / ekf_velocity_update / ekfslam_step(alphas)).

f is MotionModel.moveWithoutNoise, pinned bit-exactly to the reference's
outputs (tests/golden/motion.npz, test_oracle_rows); its Jacobians and the
process noise V M V^T are checked on the CPU (central differences, sampled
moveWithNoise).  No reference run combines the velocity model with the EKF:
parity of the combination is against the restatement only (unpinned).

Bars: batched 3-state filters and the drop-in, x_hat and P within 1e-10
relative over 60 steps (device sin/cos vs glibc, LU vs cofactor inverse);
EKF-SLAM mu within 1e-9, P within 1e-9 of max |P|, as the linear-model test.
"""
import numpy as np
import pytest

import ekf_oracle as eo

pytestmark = pytest.mark.gpu

ALPHAS = (0.1, 0.1, 0.1, 0.1, 0.1, 0.1)


@pytest.mark.parametrize("batch", [1, 4096])
def test_batched_velocity_ekf_matches_oracle(batch):
    from slamhip.ekf import DeviceEKF
    p = eo.EKFParams()
    rs = np.random.RandomState(batch + 7)
    steps = 60
    x0 = p.x0 + rs.normal(0, 0.1, (batch, 3))
    dev = DeviceEKF(batch, motion="velocity", alphas=ALPHAS)
    try:
        dev.set_state(x0, np.repeat(p.p0.reshape(1, 9), batch, 0))
        t = np.arange(1, steps + 1) * p.dt * p.omega
        base = np.stack([10 * np.cos(t), 10 * np.sin(t)], 1)
        z_all = base[:, None, :] + rs.normal(0, 1.0, (steps, batch, 2))
        xh = dev.run(z_all)
        xs, Ps = dev.get_state()
    finally:
        dev.close()
    check = range(batch) if batch <= 64 else rs.choice(batch, 100, replace=False)
    for b in check:
        x, P = x0[b].copy(), p.p0.copy()
        for s in range(steps):
            _, x, P = eo.ekf_velocity_update(x, P, z_all[s, b], p, (p.vel, p.omega), ALPHAS)
            np.testing.assert_allclose(xh[s, b], x, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(Ps[b], P, rtol=1e-10, atol=1e-15)


def test_dropin_velocity_step_with_controls():
    from extended_kalman_filter import ExtendedKalmanFilter
    p = eo.EKFParams()
    alphas = (0.2, 0.05, 0.1, 0.2, 0.05, 0.1)
    ekf = ExtendedKalmanFilter(100, motion="velocity", alphas=alphas)
    x, P = p.x0.copy(), p.p0.copy()
    rs = np.random.RandomState(11)
    for s in range(60):
        ctl = (p.vel * (1 + 0.3 * np.sin(s)), p.omega * (1 + 0.5 * np.cos(s)))
        z = x[:2] + rs.normal(0, 1, 2)
        xh, Pg = ekf.step(ctl, z.reshape(2, 1))
        _, x, P = eo.ekf_velocity_update(x, P, z, p, ctl, alphas)
        np.testing.assert_allclose(xh[:, 0], x, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(Pg, P, rtol=1e-10, atol=1e-15)


def test_velocity_prediction_is_not_the_linear_one():
    """The two motion options really differ (the option reaches the kernel)."""
    from slamhip.ekf import DeviceEKF
    p = eo.EKFParams()
    z = np.array([[10.0, 0.2]])
    out = []
    for m in ("linear", "velocity"):
        dev = DeviceEKF(1, motion=m)
        try:
            out.append(dev.step(z, control=(1.0, 0.4)))
        finally:
            dev.close()
    assert not np.allclose(out[0][0], out[1][0])


def _slam_world(n_lm, seed):
    rs = np.random.RandomState(seed)
    lm = np.column_stack([rs.uniform(-30, 30, (n_lm, 2)), rs.uniform(-np.pi, np.pi, n_lm)])
    mu = np.concatenate([[0.0, 0.0, 0.3], (lm + rs.normal(0, 0.2, lm.shape)).ravel()])
    n = mu.size
    A = rs.normal(0, 0.02, (n, n // 3 + 1))
    P = A @ A.T + np.diag(np.concatenate([[0.01, 0.01, 0.002], np.full(n - 3, 0.04)]))
    P = 0.5 * (P + P.T)
    return rs, lm, mu, P


@pytest.mark.parametrize("n_lm,k,steps", [(50, 8, 10), (300, 20, 4)])
def test_ekfslam_velocity_matches_oracle(n_lm, k, steps):
    from slamhip.ekf import DeviceEKFSLAM
    rs, lm, mu, P = _slam_world(n_lm, n_lm + 1)
    dt = 0.1
    q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
    noise = (0.05, np.deg2rad(2.0), np.deg2rad(2.0))
    dev = DeviceEKFSLAM(n_lm, dt=dt, q_robot=q, noise=noise, motion="velocity", alphas=ALPHAS)
    try:
        dev.set_state(mu, P)
        xr = mu[:3].copy()
        for s in range(steps):
            ctl = (1.0 + 0.1 * s, 0.3 - 0.02 * s)      # omega away from 0 (no guard in :64-86)
            xr = eo.velocity_motion(xr, *ctl, dt)
            ids = rs.choice(n_lm, k, replace=False)
            obs = np.array([eo.scan_predict(xr, lm[j]) for j in ids])
            obs[:, 0] *= 1 + rs.normal(0, 0.01, k)
            obs[:, 1:] += rs.normal(0, 0.01, (k, 2))
            dev.step(ctl, ids, obs)
            mu, P = eo.ekfslam_step(mu, P, ctl, ids, obs, dt, q, noise, alphas=ALPHAS)
            mu_g, P_g = dev.get_state()
            scale = np.abs(P).max()
            np.testing.assert_allclose(mu_g, mu, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(P_g, 0.5 * (P + P.T), rtol=0, atol=1e-9 * scale)
    finally:
        dev.close()


def test_ekfslam_velocity_predict_only():
    from slamhip.ekf import DeviceEKFSLAM
    n_lm = 130
    rs, lm, mu, P = _slam_world(n_lm, 2)
    dev = DeviceEKFSLAM(n_lm, motion="velocity", alphas=ALPHAS)
    try:
        dev.set_state(mu, P)
        ctl = (0.7, -0.2)
        dev.predict(ctl)
        mu_g, P_g = dev.get_state()
        mu_o, P_o = eo.ekfslam_predict(mu, P, ctl, 0.1, None, alphas=ALPHAS)
        np.testing.assert_allclose(mu_g, mu_o, rtol=1e-14, atol=1e-15)
        np.testing.assert_allclose(P_g, 0.5 * (P_o + P_o.T), rtol=1e-12, atol=1e-16)
    finally:
        dev.close()
