"""CPU checks of the oracle's O(n m) EKF-SLAM row form against its dense
restatement (the C4 GPU test compares the device with the row form)."""
import numpy as np

import ekf_oracle as eo


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
