"""2-D frame conventions of the reference (mylib/transform.py:12-59).

The robot frame has +y pointing along the heading (BASE_ANG = pi/2) and +x to
the right.  Host-side helpers for world simulation; the particle kernels
evaluate the same transform on the device (csrc/pf_kernels.inl).
"""
import numpy as np

BASE_ANG = np.pi / 2.0


def _rotation(angle):
    c, s = np.cos(angle), np.sin(angle)
    return np.array([[c, -s], [s, c]])


def world2robot(origin, world):
    """world (n,2) -> frame of the pose origin (3,1)."""
    offset = world - origin.T[0, 0:2]
    return (_rotation(BASE_ANG - origin[2, 0]) @ offset.T).T


def robot2world(origin, robot):
    """robot-frame points (n,2) of the pose origin (3,1) -> world (n,2)."""
    return (_rotation(origin[2, 0] - BASE_ANG) @ robot.T).T + origin.T[0, 0:2]
