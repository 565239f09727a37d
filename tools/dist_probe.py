"""Phase timing of the sharded step's kernels (development tool): the bench's
N = 1 sharded workload through a probe build (tools/build_variant.sh probe
-DSLAM_PROBE); prints, per batch, the wall-clock phases (us) of
dist_resample_merged_kernel (last resample step) and dist_reduce_kernel (last
step)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
os.environ.setdefault("SLAM_HIP_LIB", os.path.join(ROOT, "slam-robot_simu_amd/slamhip/libslam_probe.so"))
if len(sys.argv) > 1:
    os.environ["SLAM_HIP_LIB"] = os.path.join(ROOT, f"slam-robot_simu_amd/slamhip/libslam_{sys.argv[1]}.so")
import bench  # noqa: E402
from slamhip.dist import DistFilter  # noqa: E402

lib = C.CDLL(os.environ["SLAM_HIP_LIB"])
buf = (C.c_ulonglong * 32)()
steps = 8
lm, zs, (vel, omega, dt) = bench.simulate_world(10 * steps)
ctl = np.tile([vel, omega], (10 * steps, 1))
f = DistFilter(bench.NP_PER_GPU, lm, world=1, dt=dt, motion="velocity", likelihood="logsum", seed=3)
f.load_observations(zs)
tick = 0.01      # wall_clock64: 100 MHz
for r in range(10):
    lib.slam_probe_read(buf, 32)
    try:
        out = f.run(r * steps, ctl[r * steps:(r + 1) * steps])
    except Exception as e:            # experiment builds may break the exchange on purpose
        print("run:", e)
        out = []
    lib.slam_probe_read(buf, 32)
    t = list(buf)
    d = lambda a, b: (t[b] - t[a]) * tick if t[a] and t[b] else float("nan")
    print(f"batch {r}: resample A {d(16, 17):6.2f} scans {d(17, 18):5.2f} push {d(18, 19):5.2f} "
          f"wait {d(19, 20):5.2f} fold {d(20, 21):5.2f} rel {d(21, 22):5.2f} | B {d(22, 23):6.2f} "
          f"relB {d(23, 24):5.2f} | C {d(24, 25):6.2f} sig {d(25, 26):5.2f} | total(to signal) {d(16, 26):6.2f} || "
          f"reduce: rec[ld {d(27, 0):5.2f} red {d(0, 1):5.2f} cand {d(1, 2):5.2f} misc {d(2, 3):5.2f} win {d(3, 28):5.2f}] record {d(27, 28):5.2f} push {d(28, 29):5.2f} wait {d(29, 30):5.2f} "
          f"finalize {d(30, 31):5.2f} total {d(27, 31):6.2f}  resampled {sum(o['resampled'] for o in out)} "
          f"selected {t[15]}")
f.close()
