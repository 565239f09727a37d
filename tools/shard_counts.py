"""Development probe: the resample exchange volume of the sharded filter
(BASELINE config 3 form, in-process shards on one GPU).  Prints, per resample
step, the item counts each source shard sends to each destination shard
(items = distinct resampled particles with their destination range)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from slamhip.shard import DeviceShard, LocalComm, ShardedFilter  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n_local = 1 << 20
steps = 30
lm, zs, (vel, om, dt) = bench.simulate_world(steps)
shards = [DeviceShard(n_local, world * n_local, r * n_local, lm, dt=dt, motion="velocity",
                      likelihood="logsum", seed=77) for r in range(world)]
rec = []
orig = DeviceShard.plan


def plan(self, gb):
    c = orig(self, gb)
    rec.append(c.copy())
    return c


DeviceShard.plan = plan
filt = ShardedFilter(shards, list(range(world)), LocalComm(world), world * n_local)
for k in range(steps):
    rec.clear()
    o = filt.step((vel, om), zs[k])
    if rec:
        m = np.array(rec)
        off = m.copy()
        np.fill_diagonal(off, 0)
        print(f"step {k:2d} resample: max off-diagonal items {off.max():7d}  total off {off.sum():8d}"
              f"  self max {np.diag(m).max():7d}  ess {o['ess']:.0f}")
filt.close()
