"""First-batch penalty of DeviceParticleFilter.run (development probe): the
bench's order (create, load, prepare_graphs, 5 warm-up steps) then run(20)
three times and run(50) twice, each timed; with PRIME=<steps>, that many
untimed steps first (device clocks up before the warm-up)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

prime = int(os.environ.get("PRIME", "0"))
plan = [20, 20, 20, 50, 50]
total = prime + 5 + sum(plan)
lm, zs, (vel, omega, dt) = bench.simulate_world(total)
ctl = np.tile([vel, omega], (total, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
pf.load_observations(zs)
pf.prepare_graphs()
s = 0
if prime:
    t0 = time.perf_counter()
    pf.run(0, ctl[:prime], want_results=False)
    print(f"prime {prime} steps: {(time.perf_counter() - t0) * 1e3:.2f} ms")
    s = prime
pf.run(s, ctl[s:s + 5], want_results=False)
s += 5
for k in plan:
    t0 = time.perf_counter()
    out = pf.run(s, ctl[s:s + k])
    el = time.perf_counter() - t0
    print(f"PRIME={prime} run({k}) from {s}: {el / k * 1e3:.4f} ms/step  resamples {sum(o['resampled'] for o in out)}")
    s += k
