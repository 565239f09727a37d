"""Fused-kernel time against the landmark count (development tool): the slope
is the per-update cost, the intercept the per-particle cost of predict, RNG,
exp and the block epilogue."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
from slamhip.pf import DeviceParticleFilter  # noqa: E402

n = 1 << 20
steps = 16
rs = np.random.RandomState(1)
for nl in [int(v) for v in os.environ.get("NLS", "1 25 50 100 200").split()]:
    lm = rs.uniform(-10, 10, (nl, 2))
    zs = rs.uniform(-10, 10, (2 * steps, nl, 2))
    ctl = np.tile([1.745, 0.1745], (2 * steps, 1))
    pf = DeviceParticleFilter(n, lm, dt=0.1, motion="velocity", likelihood="logsum", seed=3)
    pf.load_observations(zs)
    pf.run(0, ctl[:steps], want_results=False)
    pf.enable_timing(True)
    pf.run(steps, ctl[steps:])
    f = pf.timing(0)
    print(f"NL={nl:4d}: fused {f[0] / f[1] * 1e3:7.2f} us  ({n * nl / (f[0] / f[1] * 1e-3):.3e} upd/s)",
          flush=True)
    pf.close()
