"""Per-step diff of finscan vs separate launches (debug aid)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "slam-robot_simu_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import pf_oracle as po
from slamhip.pf import DeviceParticleFilter

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
rs = np.random.RandomState(4)
nl, steps = 100, 24
lm = rs.uniform(-10, 10, (nl, 2))
p = po.PFParams(n_particles=n, landmarks=lm, motion="velocity")
world = po.PFWorld(p)
np.random.seed(11)
zs = []
for _ in range(steps):
    world.advance()
    zs.append(world.observe())
ctl = np.tile([p.vel, p.omega], (steps, 1))
outs = []
for fin in (True, False):
    with DeviceParticleFilter(n, lm, motion="velocity", seed=5) as d:
        d.set_finscan(fin)
        d.load_observations(np.array(zs))
        outs.append(d.run(0, ctl))
for k, (a, b) in enumerate(zip(*outs)):
    diffs = []
    for key in a:
        va, vb = np.asarray(a[key]), np.asarray(b[key])
        if not np.array_equal(va, vb):
            diffs.append(f"{key}: {va.ravel()[:9]} vs {vb.ravel()[:9]}")
    print(k, "resampled", a["resampled"], b["resampled"], "OK" if not diffs else "DIFF")
    for dd in diffs:
        print("   ", dd)
