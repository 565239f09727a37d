"""Phase timing of the resample passes (development tool): runs the C2
workload through a probe build (tools/build_variant.sh probe -DSLAM_PROBE) and
prints, for the last resample step of each batch, the wall-clock phases of the
exact cumsum (classify, ticket, tile-total scans, place + fold, release, c
stored, inverse map) in microseconds: scan_lean_merged_kernel at 2^20, the
two-launch form (plus its expand pass's own classification) above.

    python tools/scan_probe.py [NP]        (default the bench's 2^20)

The max stamps sample every 32nd workgroup (pf_kernels.inl PROBE_MAX): one
word taking every workgroup's atomic would serialise them and time itself."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
os.environ.setdefault("SLAM_HIP_LIB", os.path.join(ROOT, "slam-robot_simu_amd/slamhip/libslam_probe.so"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

lib = C.CDLL(os.environ["SLAM_HIP_LIB"])
buf = (C.c_ulonglong * 32)()
steps = 8
lm, zs, (vel, omega, dt) = bench.simulate_world(10 * steps)
ctl = np.tile([vel, omega], (10 * steps, 1))
NP = int(sys.argv[1]) if len(sys.argv) > 1 else bench.NP_PER_GPU
pf = DeviceParticleFilter(NP, lm, dt=dt, motion="velocity", likelihood="logsum", seed=3)
pf.load_observations(zs)
tick_us = 0.01      # wall_clock64: 100 MHz
for r in range(10):
    out = pf.run(r * steps, ctl[r * steps:(r + 1) * steps])
    lib.slam_probe_read(buf, 32)
    t = list(buf)
    if t[1] == 0:
        print(f"batch {r}: no resample")
        continue
    d = lambda a, b: (t[b] - t[a]) * tick_us
    print(f"batch {r}: classify {d(0, 12):6.2f}  ticket {d(12, 1):5.2f}  scans {d(1, 2):5.2f}  "
          f"place+fold {d(2, 4):5.2f}  release {d(4, 5):5.2f} | expand: c {d(5, 6):6.2f}  "
          f"inverse {d(6, 7):5.2f}  | total {d(0, 7):6.2f}  nspecial {out[-1].get('n_special', '?')}"
          + (f" | expand classify {d(5, 9):6.2f} c {d(9, 6):6.2f}" if t[9] else ""))
