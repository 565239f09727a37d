"""Round-6 probe (development tool): at C2 (2^20 x 100, velocity, logsum) the
fused kernel's event time with the device Philox normals (the bench's
instantiation) against the same kernel reading pre-drawn normals
(HOSTNOISE, particle-major [n][3]: the noise a separate kernel would stage),
and the step / finalize / scan times of each; then the bench-style graph run."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

n, steps = bench.NP_PER_GPU, 40
lm, zs, (vel, omega, dt) = bench.simulate_world(700)
ctl = np.tile([vel, omega], (700, 1))
g = np.random.RandomState(0).standard_normal((n, 3))
for mode in ("philox", "host", "philox", "host"):
    pf = DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum", seed=3)
    pf.load_observations(zs)
    pf.run(0, ctl[:62], want_results=False)
    pf.enable_timing(True)
    for k in range(steps):
        z = zs[62 + k]
        u = 0.5 if pf.resample_next else float("nan")
        pf.step((vel, omega), z, g if mode == "host" else None, u)
    t = [pf.timing(k) for k in range(4)]
    pf.close()
    print(f"{mode:7s} fused {t[0][0] / t[0][1] * 1e3:6.2f} us  finalize {t[1][0] / max(t[1][1], 1) * 1e3:6.2f} us  "
          f"scan {t[2][0] / max(t[2][1], 1) * 1e3:6.2f} us ({t[2][1]} launches)  step {t[3][0] / t[3][1] * 1e3:6.2f} us", flush=True)
pf = DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
pf.load_observations(zs)
pf.prepare_graphs()
bench.settle(pf.run, ctl, 620)
for r in range(3):
    t0 = time.perf_counter()
    out = pf.run(620 + 20 * r, ctl[620 + 20 * r:640 + 20 * r])
    el = time.perf_counter() - t0
    print(f"graph run 20 steps: {el / 20 * 1e3:.4f} ms/step  resamples {sum(o['resampled'] for o in out)}")
