"""Per-call overhead of DeviceParticleFilter.run (development probe): after
prepare_graphs and a 5-step warm-up, time run(k) for several k, each twice,
and fit time = F + k c (BASELINE configs[1] workload)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

ks = [8, 20, 8, 20, 50, 50, 1, 1, 9, 16]
total = 5 + sum(ks)
lm, zs, (vel, omega, dt) = bench.simulate_world(total)
ctl = np.tile([vel, omega], (total, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=3)
pf.load_observations(zs)
print("capture ms", pf.prepare_graphs())
pf.run(0, ctl[:5], want_results=False)
s = 5
rows = []
for k in ks:
    t0 = time.perf_counter()
    out = pf.run(s, ctl[s:s + k])
    el = time.perf_counter() - t0
    rows.append((k, el * 1e3, sum(o["resampled"] for o in out)))
    print(f"run({k:2d}) from step {s:3d}: {el * 1e3:.3f} ms  {el / k * 1e3:.4f} ms/step  resamples {rows[-1][2]}")
    s += k
k = np.array([r[0] for r in rows[2:6]], float)
t = np.array([r[1] for r in rows[2:6]])
c, F = np.polyfit(k, t, 1)
print(f"fit (calls 3-6): {c:.4f} ms/step + {F * 1e3:.1f} us per call")
