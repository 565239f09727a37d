"""Fused-kernel / step A/B over library variants (development tool, round 6):
for each library (argv; 'default' = the product build) the C2 bench workload
(graphs, 620 settle steps, 50 timed steps) and a kernel-timing pass, the
variants interleaved round-robin for `--rounds` rounds in ONE process per
round-robin pass so that box-to-box variance cancels; then the fused kernel's
event time against the particle count (intercept = the launch's fixed cost)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time
import numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, os.path.join(%(root)r, "slam-robot_simu_amd"))
import bench
from slamhip.pf import DeviceParticleFilter
n = int(os.environ.get("AB_N", str(1 << 20)))
steps = 50
lm, zs, (vel, omega, dt) = bench.simulate_world(620 + 3 * steps)
ctl = np.tile([vel, omega], (620 + 3 * steps, 1))
pf = DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
if os.environ.get("AB_SEED_NOISE") == "1":        # HBM-noise probe: h->noise holds real normals
    pf.step((vel, omega), zs[0], np.random.RandomState(0).standard_normal((n, 3)))
pf.load_observations(zs)
pf.prepare_graphs()
bench.settle(pf.run, ctl, 620)
t0 = time.perf_counter()
out = pf.run(620, ctl[620:620 + steps])
el = time.perf_counter() - t0
pf.enable_timing(True)
pf.run(620 + steps, ctl[620 + steps:620 + 2 * steps])
t = [pf.timing(k) for k in range(4)]
f = lambda k: t[k][0] / max(t[k][1], 1) * 1e3
print(f"RESULT {os.environ.get('SLAM_HIP_LIB', 'default').split('/')[-1]} n={n}: step {el / steps * 1e3:.4f} ms "
      f"fused {f(0):.2f} us finalize {f(1):.2f} us scan {f(2):.2f} us resamples {sum(o['resampled'] for o in out)}",
      flush=True)
'''


def main():
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = 2
    for a in sys.argv[1:]:
        if a.startswith("--rounds="):
            rounds = int(a.split("=")[1])
    sizes = [int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--n=")]
    code = CHILD % {"root": ROOT}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ)
            env["AB_SEED_NOISE"] = "1" if lib == "hbmnoise" else "0"
            if lib != "default":
                env["SLAM_HIP_LIB"] = os.path.join(ROOT, "slam-robot_simu_amd/slamhip", f"libslam_{lib}.so")
            for n in sizes or [1 << 20]:
                env["AB_N"] = str(n)
                subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)


if __name__ == "__main__":
    main()
