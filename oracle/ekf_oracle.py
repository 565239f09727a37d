"""ORACLE -- test infrastructure only.

CPU (NumPy) restatement of the reference EKF localisation step
(extended_kalman_filter.py) and of the EKF-SLAM extension named by
BASELINE.json config 4.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it.

Pinned: ``EKFOracle`` reproduces tests/golden/ekf.npz (360 steps of the
reference main_ekf, seed 3) bit-exactly on the fixture machine.
``ekfslam_*`` has NO reference counterpart (the reference has no EKF-SLAM):
parity for it is against this restatement only -- "parity unpinned" by the
reference.  Its measurement model is the ScanSensor range/bearing/orientation
model of graph_based_slam.py:150-153 with the covariance of :187-194.
"""
from __future__ import annotations

import numpy as np

from pf_oracle import HALF_PI, motion_velocity_exact, to_world_frame, wrap_angle


class EKFParams:
    """extended_kalman_filter.py:29-84."""

    def __init__(self, period_ms=100):
        self.dt = period_ms / 1000
        self.omega = np.deg2rad(10.0)
        self.vel = 10.0 * self.omega
        self.c = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]])
        self.q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
        self.r = np.diag([1.0, 1.0]) ** 2
        self.x0 = np.array([10.0, 0.0, np.deg2rad(90.0)])
        self.p0 = np.diag([0.01, 0.01, np.deg2rad(30.0)]) ** 2


def ekf_motion(x, dt, vel, omega):
    """extended_kalman_filter.py:160-178 for one (3,) state."""
    a = dt * np.cos(x[2])
    b = dt * np.sin(x[2])
    return np.array([x[0] + vel * a, x[1] + vel * b, wrap_angle(x[2] + omega * dt)])


def ekf_jacobian(x, dt, vel):
    """extended_kalman_filter.py:180-194."""
    return np.array([[1.0, 0.0, -dt * vel * np.sin(x[2])],
                     [0.0, 1.0, dt * vel * np.cos(x[2])],
                     [0.0, 0.0, 1.0]])


# ----------------------------------------------- velocity motion model (N1)
def velocity_motion(x, v, om, dt):
    """f = MotionModel.moveWithoutNoise (motion_model.py:64-86) for one (3,)
    state -- pf_oracle.motion_velocity_exact, pinned to tests/golden/motion.npz."""
    return np.array(motion_velocity_exact(x, v, om, dt))


def velocity_jacobians(x, v, om, dt):
    """Jacobians of moveWithoutNoise (Thrun, Probabilistic Robotics, eq. 7.8 /
    7.11) at the previous estimate: G = d f / d(x, y, yaw) (only column 2 is
    not the identity's) and V = d f / d(v, omega).  t1 = the wrapped heading
    motion_model.py:79-80 forms (sin / cos are 2 pi periodic, so the wrap
    does not change them)."""
    a = v / om
    b = wrap_angle(om * dt)
    t0 = x[2]
    t1 = wrap_angle(t0 + b)
    s0, c0, s1, c1 = np.sin(t0), np.cos(t0), np.sin(t1), np.cos(t1)
    g02 = a * (-c0 + c1)
    g12 = a * (-s0 + s1)
    v00 = (-s0 + s1) / om
    v10 = (c0 - c1) / om
    v01 = (v * (s0 - s1)) / (om * om) + ((v * c1) * dt) / om
    v11 = (-(v * (c0 - c1))) / (om * om) + ((v * s1) * dt) / om
    G = np.array([[1.0, 0.0, g02], [0.0, 1.0, g12], [0.0, 0.0, 1.0]])
    V = np.array([[v00, v01], [v10, v11], [0.0, dt]])
    return G, V


def velocity_process_noise(v, om, dt, alphas):
    """The state-space process noise of moveWithNoise (motion_model.py:31-62):
    V M V^T with M = diag(sv^4, sw^4) -- the reference hands sigma**2 to
    np.random.normal as the STANDARD DEVIATION (:46-47), so the variances are
    sigma^4 -- plus the heading noise of gamma-hat, std sg^2, entering as
    gamma dt (:48, :56): variance (sg^2 dt)^2 on the yaw."""
    a1, a2, a3, a4, a5, a6 = alphas
    v2, w2 = v ** 2, om ** 2
    sv = (a1 * v2) + (a2 * w2)
    sw = (a3 * v2) + (a4 * w2)
    sg = (a5 * v2) + (a6 * w2)
    mv, mw = (sv ** 2) ** 2, (sw ** 2) ** 2
    mg = ((sg ** 2) * dt) ** 2
    return mv, mw, mg


def velocity_predict(x, P, v, om, dt, alphas):
    """EKF prediction driven by motion_model.py: x_m = f(x), P_m = G P G^T +
    V M V^T (+ the gamma term).  Operation order of ekf_kernels.inl."""
    xm = velocity_motion(x, v, om, dt)
    G, V = velocity_jacobians(x, v, om, dt)
    mv, mw, mg = velocity_process_noise(v, om, dt, alphas)
    Qv = np.array([[V[0, 0] * V[0, 0] * mv + V[0, 1] * V[0, 1] * mw,
                    V[0, 0] * V[1, 0] * mv + V[0, 1] * V[1, 1] * mw, V[0, 1] * dt * mw],
                   [0.0, V[1, 0] * V[1, 0] * mv + V[1, 1] * V[1, 1] * mw, V[1, 1] * dt * mw],
                   [0.0, 0.0, dt * dt * mw + mg]])
    Qv[1, 0], Qv[2, 0], Qv[2, 1] = Qv[0, 1], Qv[0, 2], Qv[1, 2]
    Pm = (G @ P @ G.T) + Qv
    return xm, Pm, G, Qv


def ekf_velocity_update(x_hat, P, z, p: EKFParams, control, alphas):
    """N1: the reference's EKF step (extended_kalman_filter.py:108-128) with
    the prediction taken from motion_model.py (velocity_predict) instead of
    the linear __f / jacobF / Q; the update (position fix C, inv(S), (I - G C)
    P_m) is the reference's.  Returns (x_hat_m, x_hat, P).  No reference run
    combines the two: parity unpinned except f (motion.npz)."""
    v, om = control
    xm, Pm, _, _ = velocity_predict(x_hat, P, v, om, p.dt, alphas)
    return _ekf_correct(xm.reshape(3, 1), Pm, z, p)


def _ekf_correct(xm, Pm, z, p):
    e = z.reshape(2, 1) - (p.c @ xm)
    S = (p.c @ Pm @ p.c.T) + p.r
    G = (Pm @ p.c.T) @ np.linalg.inv(S)
    xh = xm + (G @ e)
    xh[2, 0] = wrap_angle(xh[2, 0])
    Pn = (np.identity(3) - G @ p.c) @ Pm
    return xm[:, 0], xh[:, 0], Pn


def ekf_update(x_hat, P, z, p: EKFParams, control=None):
    """extended_kalman_filter.py:108-128.  Returns (x_hat_m, x_hat, P)."""
    v, om = (p.vel, p.omega) if control is None else control
    xm = ekf_motion(x_hat, p.dt, v, om).reshape(3, 1)
    F = ekf_jacobian(x_hat, p.dt, v)
    Pm = (F @ P @ F.T) + p.q
    e = z.reshape(2, 1) - (p.c @ xm)
    S = (p.c @ Pm @ p.c.T) + p.r
    G = (Pm @ p.c.T) @ np.linalg.inv(S)
    xh = xm + (G @ e)
    xh[2, 0] = wrap_angle(xh[2, 0])
    Pn = (np.identity(3) - G @ p.c) @ Pm
    return xm[:, 0], xh[:, 0], Pn


class EKFWorld:
    """Truth / observation / dead reckoning of main_ekf (:97-106)."""

    def __init__(self, p: EKFParams):
        self.p = p
        self.x_true = p.x0.copy()
        self.x_dr = p.x0.copy()

    def advance(self):
        p = self.p
        self.x_true = ekf_motion(self.x_true, p.dt, p.vel, p.omega)
        w = np.random.multivariate_normal([0.0, 0.0], p.r, 1).T          # :100
        y_l = (p.c @ np.array([[0.0], [0.0], [np.deg2rad(90.0)]])) + w     # :141-144
        z = to_world_frame(self.x_true, y_l.T).T[:, 0]                     # :145-146
        v = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, 1).T       # :105
        self.x_dr = ekf_motion(self.x_dr, p.dt, p.vel, p.omega) + v[:, 0]
        return z


def run_reference_order(seed: int, steps: int, period_ms=100):
    np.random.seed(seed)
    p = EKFParams(period_ms)
    world = EKFWorld(p)
    x_hat, P = p.x0.copy(), p.p0.copy()
    rows = []
    for _ in range(steps):
        z = world.advance()
        xm, x_hat, P = ekf_update(x_hat, P, z, p)
        rows.append(dict(x_true=world.x_true.copy(), x_dr=world.x_dr.copy(), z=z,
                         x_hat_m=xm, P=P.copy(), x_hat=x_hat.copy()))
    return rows


# ------------------------------------------------------------- EKF-SLAM
def scan_cov(dist, r_dist, r_dir, r_orient):
    """graph_based_slam.py:187-194 measurement covariance (range, bearing, orientation)."""
    d = dist * r_dist
    return np.diag([d ** 2, (dist * np.sin(r_dir)) ** 2, r_dir ** 2 + r_orient ** 2])


def scan_predict(xr, lm):
    """graph_based_slam.py:150-153: landmark (x, y, phi) seen from pose xr ->
    (range, bearing, orientation).  Orientation follows the sensor's
    convention ``BASE_ANG - yaw`` plus the landmark's own heading phi."""
    c, s = np.cos(HALF_PI - xr[2]), np.sin(HALF_PI - xr[2])
    dx, dy = lm[0] - xr[0], lm[1] - xr[1]
    rx = c * dx - s * dy
    ry = s * dx + c * dy
    return np.array([np.hypot(rx, ry), np.arctan2(ry, rx), wrap_angle(HALF_PI - xr[2] + lm[2])])


def scan_jacobian(xr, lm):
    """d(range, bearing, orientation) / d(robot x,y,yaw ; landmark x,y,phi)."""
    dx, dy = lm[0] - xr[0], lm[1] - xr[1]
    q = dx * dx + dy * dy
    r = np.sqrt(q)
    Hr = np.array([[-dx / r, -dy / r, 0.0],
                   [dy / q, -dx / q, -1.0],
                   [0.0, 0.0, -1.0]])
    Hl = np.array([[dx / r, dy / r, 0.0],
                   [-dy / q, dx / q, 0.0],
                   [0.0, 0.0, 1.0]])
    return Hr, Hl


def ekfslam_predict(mu, P, control, dt, q_robot, alphas=None):
    """EKF-SLAM prediction on the robot rows / columns: the reference EKF's
    linear model (:160-194, + q_robot), or with ``alphas`` the velocity model
    of motion_model.py (moveWithoutNoise, G, V M V^T: velocity_predict)."""
    v, om = control
    mu = mu.copy()
    xr = mu[:3].copy()
    P = P.copy()
    if alphas is None:
        F = ekf_jacobian(xr, dt, v)
        mu[:3] = ekf_motion(xr, dt, v, om)
        Q = q_robot
    else:
        _, _, F, Q = velocity_predict(xr, P[:3, :3], v, om, dt, alphas)
        mu[:3] = velocity_motion(xr, v, om, dt)
    P[:3, :] = F @ P[:3, :]
    P[:, :3] = P[:, :3] @ F.T
    P[:3, :3] += Q
    return mu, P


def ekfslam_step(mu, P, control, obs_ids, obs, dt, q_robot, noise, alphas=None):
    """One EKF-SLAM predict + batched update.

    mu (n,), P (n,n) with n = 3 + 3*NLM; robot motion = the reference EKF's
    linear model (:160-194), or motion_model.py's velocity model with
    ``alphas`` (ekfslam_predict); ``obs`` (k,3) range/bearing/orientation of
    the landmarks ``obs_ids``; ``noise`` = (r_dist, r_dir, r_orient).  The
    update is P <- P - K S K^T with K = P H^T S^-1 (rank-3k)."""
    n = mu.size
    mu, P = ekfslam_predict(mu, P, control, dt, q_robot, alphas)
    k = len(obs_ids)
    H = np.zeros((3 * k, n))
    innov = np.zeros(3 * k)
    Rb = np.zeros((3 * k, 3 * k))
    for t, (j, o) in enumerate(zip(obs_ids, obs)):
        sl = slice(3 + 3 * j, 6 + 3 * j)
        zhat = scan_predict(mu[:3], mu[sl])
        Hr, Hl = scan_jacobian(mu[:3], mu[sl])
        H[3 * t:3 * t + 3, :3] = Hr
        H[3 * t:3 * t + 3, sl] = Hl
        e = o - zhat
        e[1] = wrap_angle(e[1])
        e[2] = wrap_angle(e[2])
        innov[3 * t:3 * t + 3] = e
        Rb[3 * t:3 * t + 3, 3 * t:3 * t + 3] = scan_cov(o[0], *noise)
    PHt = P @ H.T
    S = H @ PHt + Rb
    K = PHt @ np.linalg.inv(S)
    mu = mu + K @ innov
    mu[2] = wrap_angle(mu[2])
    P = P - K @ S @ K.T
    return mu, P


def ekfslam_update_rows(mu, P_idx, P_rows, rows, obs_ids, obs, noise):
    """The update half of ``ekfslam_step`` evaluated on selected rows of P only
    (O(n m), for checking an n = 30,003 covariance without an n x n host copy).

    ``P_idx``: rows idx = (0, 1, 2, 3+3j, 4+3j, 5+3j for j in obs_ids) of the
    symmetric prior P (|idx| x n) -- H is non-zero only in those columns, so
    P H^T = P_idx^T H_idx^T.  ``P_rows``: the prior's rows ``rows`` (r x n).
    Returns (mu_new, P_rows_new) with P_new = P - K (P H^T)^T, K = P H^T S^-1
    (= P - K S K^T of ekfslam_step)."""
    idx = [0, 1, 2]
    for j in obs_ids:
        idx += [3 + 3 * j, 4 + 3 * j, 5 + 3 * j]
    idx = np.asarray(idx)
    k = len(obs_ids)
    m = 3 * k
    Hs = np.zeros((m, idx.size))
    innov = np.zeros(m)
    Rb = np.zeros((m, m))
    for t, (j, o) in enumerate(zip(obs_ids, obs)):
        lm = mu[3 + 3 * j:6 + 3 * j]
        zhat = scan_predict(mu[:3], lm)
        Hr, Hl = scan_jacobian(mu[:3], lm)
        Hs[3 * t:3 * t + 3, :3] = Hr
        Hs[3 * t:3 * t + 3, 3 + 3 * t:6 + 3 * t] = Hl
        e = o - zhat
        e[1] = wrap_angle(e[1])
        e[2] = wrap_angle(e[2])
        innov[3 * t:3 * t + 3] = e
        Rb[3 * t:3 * t + 3, 3 * t:3 * t + 3] = scan_cov(o[0], *noise)
    PHt = P_idx.T @ Hs.T                       # n x m
    S = Hs @ PHt[idx] + Rb
    K = PHt @ np.linalg.inv(S)
    mu = mu + K @ innov
    mu[2] = wrap_angle(mu[2])
    return mu, P_rows - K[np.asarray(rows)] @ PHt.T
