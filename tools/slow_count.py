"""Probe (SLAM_HIP_LIB = a -DSLAM_PROBE_COUNT_SLOW build): log-sum slow-path
particles and blocks per step of the bench workload."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip import _lib  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

lib = _lib.load()
steps = 30
lm, zs, (vel, omega, dt) = bench.simulate_world(steps)
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
pf.load_observations(zs)
buf = (C.c_ulonglong * 2)()
lib.slam_probe_slow_count(buf)
for k in range(steps):
    out = pf.run(k, np.array([[vel, omega]]))
    lib.slam_probe_slow_count(buf)
    print(f"step {k:2d} {'res' if out[0]['resampled'] else '   '} slow particles {buf[0]:7d} "
          f"blocks {buf[1]:5d} / 2048  ess {out[0]['ess']:.0f}")
