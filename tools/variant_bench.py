"""Kernel-variant timing (development tool): the C2 workload's fused-kernel and
step times through the library named by SLAM_HIP_LIB."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

steps = 24
lm, zs, (vel, omega, dt) = bench.simulate_world(3 * steps)
ctl = np.tile([vel, omega], (3 * steps, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity",
                          likelihood=os.environ.get("VB_LIK", "logsum"), seed=3)
pf.load_observations(zs)
pf.run(0, ctl[:steps], want_results=False)
t0 = time.perf_counter()
pf.run(steps, ctl[steps:2 * steps])
el = time.perf_counter() - t0
pf.enable_timing(True)
pf.run(2 * steps, ctl[2 * steps:])
f = pf.timing(0)
r = pf.timing(1)
s = pf.timing(2)
print(f"{os.environ.get('SLAM_HIP_LIB', 'default')}: step {el / steps * 1e3:.4f} ms  "
      f"fused {f[0] / max(f[1], 1) * 1e3:.1f} us  reduce {r[0] / max(r[1], 1) * 1e3:.1f} us  "
      f"scan {s[0] / max(s[1], 1) * 1e3:.1f} us")
