"""Drop-in MotionModel (motion_model.py:14-86) backed by the MI355X kernel
``slam_motion_velocity`` (libslam_hip.so).

Same constructor and methods as the reference:

  MotionModel(dt, a1, a2, a3, a4, a5, a6)
  moveWithNoise(aPose, aV, aW)     -- sample_motion_model_velocity (:31-62)
  moveWithoutNoise(aPose, aV, aW)  -- the noise-free motion (:64-86)

``aPose`` is a (3, 1) column as in the reference, or a (3, N) batch: column j
of a batch gives exactly what the j-th of N consecutive reference calls gives.
The noise is drawn from NumPy's global RNG in the reference's order (three
normals per call: v, w, gamma, :46-48), so a seeded run reproduces the
reference stream; the std handed to normal() is sigma**2 as in the reference
(:46-48), and ``np.random.normal(0, s)`` is ``0 + s * g`` with the same draw g
that ``standard_normal`` returns.  The motion itself runs on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from slamhip import _lib
from slamhip._lib import check, dptr


class MotionModel(object):
    """Velocity motion model (Probabilistic Robotics, ch. 5), on the GPU."""

    def __init__(self, dt, a1, a2, a3, a4, a5, a6, *, device=0):
        self.__mDt = dt                                   # :28
        self.__mNoise = (a1, a2, a3, a4, a5, a6)          # :29
        self._params = np.array([dt, a1, a2, a3, a4, a5, a6], dtype=np.float64)
        self._device = int(device)
        self._lib = _lib.load()

    def _run(self, aPose, aV, aW, normals):
        pose = np.asarray(aPose, dtype=np.float64)
        if pose.ndim != 2 or pose.shape[0] != 3:
            raise ValueError("aPose must be a (3, 1) pose or a (3, N) batch of poses")
        n = pose.shape[1]
        rows = np.ascontiguousarray(pose.T)               # n x 3 (x, y, theta)
        out = np.empty((n, 3))
        nz = None if normals is None else np.ascontiguousarray(normals, dtype=np.float64)
        check(self._lib.slam_motion_velocity(dptr(self._params), n, dptr(rows), float(aV), float(aW),
                                             dptr(nz), dptr(out), self._device),
              "slam_motion_velocity")
        return np.ascontiguousarray(out.T)

    def moveWithNoise(self, aPose, aV, aW):
        """motion_model.py:31-62 -> new pose(s), same shape as aPose."""
        n = np.asarray(aPose).shape[1]
        g = np.random.standard_normal(3 * n).reshape(n, 3)   # :46-48, call after call
        return self._run(aPose, aV, aW, g)

    def moveWithoutNoise(self, aPose, aV, aW):
        """motion_model.py:64-86 -> new pose(s), same shape as aPose."""
        return self._run(aPose, aV, aW, None)
