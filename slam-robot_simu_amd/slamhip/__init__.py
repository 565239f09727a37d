"""slamhip -- MI355X (gfx950) implementation of the SLAM-Robot_Simu estimator
hot path behind a ctypes C-ABI (include/slam_hip.h)."""
from ._lib import SlamError, device_count, load  # noqa: F401

__all__ = ["SlamError", "device_count", "load"]
