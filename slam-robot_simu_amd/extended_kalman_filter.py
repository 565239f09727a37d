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

    def __init__(self, period_ms, *, device=0, motion="linear", alphas=None):
        """motion="velocity": the filter's prediction is driven by motion_model.py
        (MotionModel.moveWithoutNoise, its Jacobian and moveWithNoise's noise
        from ``alphas`` a1..a6, default 0.1 each); "linear" is the reference's
        own __f / jacobF / Q.  The simulated truth stays the reference's."""
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
        kw = {} if alphas is None else {"alphas": alphas}
        self.dev = DeviceEKF(1, device=device, motion=motion, **kw, **p)

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


# ---------------------------------------------------------------- animation
class EKFAnimation:
    """The reference's demo frame (extended_kalman_filter.py:219-274) over
    this filter: true track, observations, predicted track and the error
    ellipse of P."""

    def __init__(self, ekf, period_ms, confidence=99.0):
        from mylib.error_ellipse import ErrorEllipse
        self.ekf = ekf
        self.period_ms = period_ms
        self.confidence = confidence
        self.ellipse = ErrorEllipse(confidence)
        self.truth, self.obs, self.pred = [], [], []
        self.time_s = 0.0

    def __call__(self, i):
        import matplotlib.pyplot as plt
        from mylib import plots
        self.time_s += self.period_ms / 1000
        x_true, x_dr, obs, x_pre, P = self.ekf.main_ekf()
        self.truth.append(x_true[0:2, :].copy())
        self.obs.append(np.asarray(obs).reshape(2, 1).copy())
        self.pred.append(x_pre[0:2, :].copy())
        plt.cla()
        ax = plt.subplot2grid((1, 1), (0, 0))
        plots.trajectory(ax, self.truth, "red", "Ground Truth")
        zs = np.concatenate(self.obs, axis=1)
        ax.scatter(zs[0], zs[1], c="green", marker="o", alpha=0.5, label="Observation")
        plots.trajectory(ax, self.pred, "blue", "Predicted")
        plots.error_ellipse(ax, (x_pre[0, 0], x_pre[1, 0]), self.ellipse, P[0:2, 0:2],
                            label="Error Ellipse: %.2f[%%]" % self.confidence)
        print("time:{0:.3f}[s], x-cov:{1:.3f}[m], y-cov:{2:.3f}[m], xy-cov:{3:.3f}[m]"
              .format(self.time_s, P[0, 0], P[1, 1], P[1, 0]))
        ax.set_aspect("equal", adjustable="datalim")
        plots.finish(ax, "Localization by EKF")
        return (ax,)


_animations = {}


def animate(i, ekf, period_ms):
    """FuncAnimation callback with the reference's signature (:219)."""
    key = id(ekf)
    if key not in _animations:
        _animations[key] = EKFAnimation(ekf, period_ms)
    return _animations[key](i)


if __name__ == "__main__":
    import matplotlib.animation as animation
    import matplotlib.pyplot as plt

    period_ms = 100
    frame_cnt = int(36 * 1000 / period_ms)
    fig = plt.figure(figsize=(12, 9))
    ekf = ExtendedKalmanFilter(period_ms)
    ani = animation.FuncAnimation(fig, animate, frames=frame_cnt, fargs=(ekf, period_ms), blit=False,
                                  interval=period_ms, repeat=False)
    plt.show()
