"""NumPy-stream step time (development A/B): bench's alt_modes.numpy_stream
measurement alone -- settle, 5 warm-up steps, 64 timed steps -- through the
library named by SLAM_HIP_LIB."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

settle, steps = 20 * bench.SETTLE_BATCH, bench.NS_ROUND_STEPS
total = settle + 5 + steps
lm, zs, (vel, om, dt) = bench.simulate_world(total)
ctl = np.tile([vel, om], (total, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
pf.use_numpy_stream(np.random.RandomState(1234))
pf.load_truth(bench.simulate_world.poses)
pf.prepare_graphs()
s0 = bench.settle(pf.run, ctl, settle)
pf.run(s0, ctl[s0:s0 + 5], want_results=False)
t0 = time.perf_counter()
pf.run(s0 + 5, ctl[s0 + 5:s0 + 5 + steps])
el = time.perf_counter() - t0
print(f"{os.path.basename(os.environ.get('SLAM_HIP_LIB', 'libslam_hip.so'))}: numpy stream "
      f"{el / steps * 1e3:.4f} ms/step")
