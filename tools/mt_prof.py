"""Profile target: the particle filter at 2^20 x 100 with NumPy's stream drawn
on the device (noise="mt19937" path), K graph-replayed steps."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
lm, zs, (vel, om, dt) = bench.simulate_world(steps + 5)
ctl = np.tile([vel, om], (steps + 5, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1)
pf.use_numpy_stream(np.random.RandomState(1234))
pf.load_truth(bench.simulate_world.poses)
pf.run(0, ctl[:5], want_results=False)
t0 = time.perf_counter()
out = pf.run(5, ctl[5:])
print(f"numpy-stream steps: {(time.perf_counter() - t0) * 1e3 / steps:.3f} ms/step, "
      f"resampled {sum(o['resampled'] for o in out)}")
