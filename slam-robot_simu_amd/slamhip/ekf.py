"""Device EKF filters: handles on libslam_hip's slam_ekf_* (batched 3-state
localisation, extended_kalman_filter.py) and slam_ekfslam_* (EKF-SLAM,
BASELINE config 4) entry points."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import EKFConfig, EKFSLAMConfig, check, dptr


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


def reference_ekf_config(period_ms=100):
    """The constants of ExtendedKalmanFilter.__init__ (extended_kalman_filter.py:29-84)."""
    dt = period_ms / 1000
    omega = np.deg2rad(10.0)
    return dict(dt=dt, vel=10.0 * omega, omega=omega,
                q=np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2,
                r=np.diag([1.0, 1.0]) ** 2,
                x0=np.array([10.0, 0.0, np.deg2rad(90.0)]),
                p0=np.diag([0.01, 0.01, np.deg2rad(30.0)]) ** 2)


_MOTIONS = {"linear": 0, "velocity": 1}
DEFAULT_ALPHAS = (0.1, 0.1, 0.1, 0.1, 0.1, 0.1)     # graph_based_slam.py:605 MotionModel(2.0, 0.1 x 6)


class DeviceEKF:
    """``batch`` independent 3-state EKFs on one GPU (batch=1: the reference's filter).

    ``motion="linear"``: the reference's prediction (extended_kalman_filter.py
    :160-194, Q).  ``motion="velocity"``: the prediction driven by
    motion_model.py (north_star) -- f = MotionModel.moveWithoutNoise, its
    Jacobian, and the process noise of moveWithNoise from ``alphas`` (a1..a6)."""

    def __init__(self, batch=1, *, device=0, motion="linear", alphas=DEFAULT_ALPHAS, **params):
        p = reference_ekf_config()
        p.update(params)
        cfg = EKFConfig()
        cfg.motion = _MOTIONS[motion]
        cfg.alphas[:] = [float(a) for a in alphas]
        self.motion = motion
        cfg.dt, cfg.vel, cfg.omega = float(p["dt"]), float(p["vel"]), float(p["omega"])
        cfg.q[:] = [float(v) for v in np.asarray(p["q"], float).ravel()]
        cfg.r[:] = [float(v) for v in np.asarray(p["r"], float).ravel()]
        cfg.x0[:] = [float(v) for v in np.asarray(p["x0"], float).ravel()]
        cfg.p0[:] = [float(v) for v in np.asarray(p["p0"], float).ravel()]
        self.batch = int(batch)
        self.params = p
        self._lib = _lib.load()
        h = C.c_void_p()
        check(self._lib.slam_ekf_create(C.byref(cfg), self.batch, int(device), C.byref(h)),
              "slam_ekf_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_ekf_destroy(self._h)
            self._h = None

    __del__ = close

    def set_state(self, x=None, P=None):
        x = None if x is None else _f64(x, (self.batch, 3))
        P = None if P is None else _f64(P, (self.batch, 9))
        check(self._lib.slam_ekf_set_state(self._h, dptr(x), dptr(P)), "slam_ekf_set_state")

    def get_state(self):
        x = np.empty((self.batch, 3))
        P = np.empty((self.batch, 3, 3))
        check(self._lib.slam_ekf_get_state(self._h, dptr(x), dptr(P)), "slam_ekf_get_state")
        return x, P

    def step(self, z, control=None):
        """One filter step; z: (batch, 2) world positions.  Returns (x_hat_m, x_hat, P)."""
        z = _f64(z, (self.batch, 2))
        ctl = None if control is None else _f64(control, (2,))
        xm = np.empty((self.batch, 3))
        xh = np.empty((self.batch, 3))
        P = np.empty((self.batch, 3, 3))
        check(self._lib.slam_ekf_step(self._h, dptr(ctl), dptr(z), dptr(xm), dptr(xh), dptr(P)),
              "slam_ekf_step")
        return xm, xh, P

    def run(self, z_all, control=None):
        """len(z_all) steps in one launch; z_all: (steps, batch, 2).  Returns x_hat (steps, batch, 3)."""
        z_all = _f64(z_all)
        steps = z_all.shape[0]
        z_all = z_all.reshape(steps, self.batch, 2)
        ctl = None if control is None else _f64(control, (2,))
        out = np.empty((steps, self.batch, 3))
        check(self._lib.slam_ekf_run(self._h, steps, dptr(ctl), dptr(z_all), dptr(out)),
              "slam_ekf_run")
        return out

    def run_device(self, n_steps, z_dev_ptr, xh_dev_ptr=None, control=None):
        """n_steps steps with observations already in device memory (pointer to
        n_steps x batch x 2 fp64); asynchronous (see synchronize)."""
        ctl = None if control is None else _f64(control, (2,))
        check(self._lib.slam_ekf_run_device(self._h, int(n_steps), dptr(ctl), C.c_void_p(z_dev_ptr),
                                            C.c_void_p(xh_dev_ptr) if xh_dev_ptr else None),
              "slam_ekf_run_device")

    def load_observations(self, z_all):
        z_all = _f64(z_all)
        steps = z_all.shape[0]
        check(self._lib.slam_ekf_load_observations(self._h, steps, dptr(z_all.reshape(steps, self.batch, 2))),
              "slam_ekf_load_observations")
        self.loaded_steps = steps

    def run_loaded(self, n_steps, control=None, keep_history=True):
        """Asynchronous: n_steps filter steps from the loaded observations."""
        ctl = None if control is None else _f64(control, (2,))
        check(self._lib.slam_ekf_run_loaded(self._h, int(n_steps), dptr(ctl), int(bool(keep_history))),
              "slam_ekf_run_loaded")

    def synchronize(self):
        check(self._lib.slam_ekf_synchronize(self._h), "slam_ekf_synchronize")


class DeviceEKFSLAM:
    """EKF-SLAM over ``n_landmarks`` landmarks (x, y, phi); covariance in HBM."""

    def __init__(self, n_landmarks, *, dt=0.1, q_robot=None, noise=(0.05, np.deg2rad(2.0),
                                                                         np.deg2rad(2.0)), device=0,
                 motion="linear", alphas=DEFAULT_ALPHAS):
        cfg = EKFSLAMConfig()
        cfg.dt = float(dt)
        cfg.motion = _MOTIONS[motion]
        cfg.alphas[:] = [float(a) for a in alphas]
        self.motion = motion
        q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2 if q_robot is None else np.asarray(q_robot)
        cfg.q_robot[:] = [float(v) for v in q.ravel()]
        cfg.r_dist, cfg.r_dir, cfg.r_orient = (float(v) for v in noise)
        self.n_lm = int(n_landmarks)
        self.n = 3 + 3 * self.n_lm
        self._lib = _lib.load()
        h = C.c_void_p()
        check(self._lib.slam_ekfslam_create(C.byref(cfg), self.n_lm, int(device), C.byref(h)),
              "slam_ekfslam_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_ekfslam_destroy(self._h)
            self._h = None

    __del__ = close

    def set_state(self, mu, P=None):
        mu = _f64(mu, (self.n,))
        P = None if P is None else _f64(P, (self.n, self.n))
        check(self._lib.slam_ekfslam_set_state(self._h, dptr(mu), dptr(P)), "slam_ekfslam_set_state")

    def init_diag(self, mu, p_diag):
        check(self._lib.slam_ekfslam_init_diag(self._h, dptr(_f64(mu, (self.n,))),
                                               dptr(_f64(p_diag, (self.n,)))),
              "slam_ekfslam_init_diag")

    def get_state(self, with_cov=True):
        mu = np.empty(self.n)
        P = np.empty((self.n, self.n)) if with_cov else None
        check(self._lib.slam_ekfslam_get_state(self._h, dptr(mu), dptr(P)), "slam_ekfslam_get_state")
        return (mu, P) if with_cov else mu

    def get_rows(self, rows):
        """Rows of the symmetric covariance (k x n) without copying all of P."""
        rows = np.ascontiguousarray(rows, dtype=np.int64).ravel()
        out = np.empty((rows.size, self.n))
        check(self._lib.slam_ekfslam_get_rows(self._h, int(rows.size),
                                              rows.ctypes.data_as(C.POINTER(C.c_int64)), dptr(out)),
              "slam_ekfslam_get_rows")
        return out

    def predict(self, control):
        check(self._lib.slam_ekfslam_predict(self._h, dptr(_f64(control, (2,)))),
              "slam_ekfslam_predict")

    def update(self, ids, obs):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        obs = _f64(obs, (ids.size, 3))
        check(self._lib.slam_ekfslam_update(self._h, int(ids.size),
                                            ids.ctypes.data_as(C.POINTER(C.c_int64)), dptr(obs)),
              "slam_ekfslam_update")

    def step(self, control, ids, obs):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        obs = _f64(obs, (ids.size, 3))
        check(self._lib.slam_ekfslam_step(self._h, dptr(_f64(control, (2,))), int(ids.size),
                                          ids.ctypes.data_as(C.POINTER(C.c_int64)), dptr(obs)),
              "slam_ekfslam_step")

    def timing(self):
        out = np.zeros(5)
        check(self._lib.slam_ekfslam_timing(self._h, dptr(out)), "slam_ekfslam_timing")
        return dict(gather_ms=out[0], inverse_ms=out[1], gain_ms=out[2], rank_update_ms=out[3])
