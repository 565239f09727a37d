"""The sharded step on one shard against the single handle (development probe,
for a kernel trace): bench's sharded1 workload, settle + 5 warm-up steps, then
50 timed steps of each; prints ms/step."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.dist import DistFilter  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

steps, settle = 50, 4 * bench.SETTLE_BATCH
total = settle + 5 + steps
lm, zs, (vel, omega, dt) = bench.simulate_world(total)
ctl = np.tile([vel, omega], (total, 1))
kw = dict(dt=dt, motion="velocity", likelihood="logsum", seed=1234)
for name in ("single", "sharded1", "single", "sharded1"):
    f = (DeviceParticleFilter(bench.NP_PER_GPU, lm, **kw) if name == "single"
         else DistFilter(bench.NP_PER_GPU, lm, world=1, **kw))
    try:
        f.load_observations(zs)
        f.prepare_graphs()
        s0 = bench.settle(f.run, ctl, settle)
        f.run(s0, ctl[s0:s0 + 5], want_results=False)
        t0 = time.perf_counter()
        out = f.run(s0 + 5, ctl[s0 + 5:s0 + 5 + steps])
        el = time.perf_counter() - t0
        print(f"{name}: {el / steps * 1e3:.4f} ms/step  resamples {sum(o['resampled'] for o in out)}")
    finally:
        f.close()
