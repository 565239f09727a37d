"""Angle wrap with the semantics of the reference's mylib/limit.py:11-26.

Host-side helper for world simulation (truth poses, observations).  The device
kernels carry their own copy (csrc/common.hpp: wrap_angle).
"""
import math

import numpy as np

_TWO_PI = np.pi * 2


def limit_angle(angle_in):
    """Wrap into [-pi, pi]: |a| reduced by repeated 2*pi subtraction, sign
    restored afterwards (so -0.0 -> 0.0, and +-pi stay +-pi)."""
    mag = np.absolute(angle_in)
    while mag > np.pi:
        mag -= _TWO_PI
    return -mag if angle_in < 0 else mag


def limit_angles(a):
    """Element-wise limit_angle over an array (same subtraction sequence)."""
    a = np.asarray(a, dtype=np.float64)
    mag = np.absolute(a)
    todo = mag > np.pi
    while todo.any():
        mag[todo] -= _TWO_PI
        todo = mag > np.pi
    return np.where(a < 0, -mag, mag)


__all__ = ["limit_angle", "limit_angles", "math"]
