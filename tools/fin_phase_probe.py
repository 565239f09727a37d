"""Phase timeline of the 2^20 finalize (development tool, round 6): runs the C2
workload through a probe build (tools/build_variant.sh finprobe -DSLAM_FIN_PROBE)
one step per batch and prints the finalize's wall-clock stamps (thread 0):
loads + np.sum rounds, the last buffer chain + rescale + candidates, the 11
sums + argmax + record, the record / counters, the next step's block prefix."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
os.environ.setdefault("SLAM_HIP_LIB", os.path.join(ROOT, "slam-robot_simu_amd/slamhip/libslam_finprobe.so"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

lib = C.CDLL(os.environ["SLAM_HIP_LIB"])
buf = (C.c_longlong * 32)()
n = int(os.environ.get("FP_N", str(1 << 20)))
lm, zs, (vel, omega, dt) = bench.simulate_world(700)
ctl = np.tile([vel, omega], (700, 1))
pf = DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum", seed=1234)
pf.load_observations(zs)
bench.settle(pf.run, ctl, 310)
names = ["loads+rounds", "chain+cand", "sums+argmax", "record", "prefix"]
rows = []
for k in range(310, 370):
    out = pf.run(k, ctl[k:k + 1])
    assert lib.slam_fin_probe_read(buf) == 0
    t = np.array(buf[:6], dtype=np.float64) * 0.01              # us (100 MHz)
    rows.append((np.diff(t), out[0]["resample_next"]))
for flag in (False, True):
    sel = [r for r, f in rows if f == flag]
    if sel:
        med = np.median(np.array(sel), axis=0)
        print(f"resample_next={flag} ({len(sel)} steps): " + "  ".join(f"{a} {b:5.2f}" for a, b in zip(names, med))
              + f"  | total {med.sum():5.2f} us")
