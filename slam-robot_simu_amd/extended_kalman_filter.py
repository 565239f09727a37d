"""Drop-in ExtendedKalmanFilter backed by the MI355X kernels (libslam_hip.so).

Same constructor and ``main_ekf()`` contract as the reference
(extended_kalman_filter.py:20 / :86-130), plus ``step(control, z)`` returning
``(x_hat (3,1), P (3,3))``.  The filter (prediction with jacobF, gain with
inv(S), update, P = (I - G C) P_m) runs on the GPU (csrc/ekf_kernels.inl);
this module simulates the ground truth, the observation and the dead
reckoning on the host, in the reference's order on NumPy's global RNG
(w ~ N(0, R) at :100, then v ~ N(0, Q) at :105), so a seeded run follows the
reference's trajectory.
"""
from __future__ import annotations

import numpy as np

from mylib import limit
from mylib import transform as tf
from slamhip.ekf import DeviceEKF, reference_ekf_config


class ExtendedKalmanFilter(object):
    """EKF localisation with a world-position sensor (GPU filter)."""

    def __init__(self, period_ms, *, device=0):
        p = reference_ekf_config(period_ms)
        self.dt = p["dt"]                                          # :29
        self.omega = p["omega"]                                    # :46
        self.vel = p["vel"]                                        # :47
        self.Q = p["q"]                                            # :62-66
        self.R = p["r"]                                            # :68-70
        self.C = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]])      # :58-60
        self.Q_act = self.Q                                        # :63 (simulated noise)
        self.R_act = self.R                                        # :71
        self.x_true = p["x0"].reshape(3, 1).copy()                 # :74-79
        self.x_dr = self.x_true.copy()
        self.dev = DeviceEKF(1, device=device, **p)

    def _f(self, x, v=None, om=None):
        """extended_kalman_filter.py:160-178 (host copy for truth / dead reckoning)."""
        v = self.vel if v is None else v
        om = self.omega if om is None else om
        yaw = x[2, 0]
        a = self.dt * np.cos(yaw)
        b = self.dt * np.sin(yaw)
        return np.array([[x[0, 0] + v * a], [x[1, 0] + v * b],
                         [limit.limit_angle(x[2, 0] + om * self.dt)]])

    def _observation(self, x, w):
        """extended_kalman_filter.py:132-147: robot-frame (0, 0) + w, to the world frame."""
        x_l = np.array([[0.0], [0.0], [np.deg2rad(90.0)]])
        y_l = (self.C @ x_l) + w
        return tf.robot2world(x, y_l.T).T

    def main_ekf(self):
        """One step of extended_kalman_filter.py:86-130.
        Returns (x_true, x_dr, z, x_hat_m, P)."""
        self.x_true = self._f(self.x_true)                                         # :97
        w = np.random.multivariate_normal([0.0, 0.0], self.R_act, 1).T             # :100
        z = self._observation(self.x_true, w)                                      # :101
        v = np.random.multivariate_normal([0.0, 0.0, 0.0], self.Q_act, 1).T        # :105
        self.x_dr = self._f(self.x_dr) + v                                         # :106
        xm, xh, P = self.dev.step(z.reshape(1, 2))                                 # :108-128
        self.x_hat = xh[0].reshape(3, 1)
        return self.x_true, self.x_dr, z, xm[0].reshape(3, 1), P[0]

    def step(self, control, observations):
        """North-star surface: control = (v, omega), observations = z (2,1) world
        position.  Returns (x_hat (3,1), P (3,3))."""
        z = np.asarray(observations, dtype=np.float64).reshape(1, 2)
        _, xh, P = self.dev.step(z, control=np.asarray(control, dtype=np.float64))
        return xh[0].reshape(3, 1), P[0]
