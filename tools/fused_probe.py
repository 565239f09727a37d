"""Phase timeline of the fused kernel (development tool): runs the C2 workload
through a probe build (tools/build_variant.sh fprobe -DSLAM_PROBE_FUSED) and
prints, for the last fused launch of a batch, the distribution over blocks of
the block start (relative to the first block's start) and of each phase
(wave 0 of the block): table staging, normals, predict (loads consumed),
likelihood, epilogue; blocks are split by start time into residency rounds."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
os.environ.setdefault("SLAM_HIP_LIB", os.path.join(ROOT, "slam-robot_simu_amd/slamhip/libslam_fprobe.so"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

lib = C.CDLL(os.environ["SLAM_HIP_LIB"])
nb = bench.NP_PER_GPU // 512
buf = (C.c_ulonglong * (nb * 8))()
steps = 8
lm, zs, (vel, omega, dt) = bench.simulate_world(6 * steps)
ctl = np.tile([vel, omega], (6 * steps, 1))
pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood="logsum", seed=3)
pf.load_observations(zs)
names = ["stage", "normals", "predict", "lik", "epilogue"]
for r in range(6):
    out = pf.run(r * steps, ctl[r * steps:(r + 1) * steps])
    assert lib.slam_fprobe_read(buf, nb * 8) == 0
    t = np.array(buf, dtype=np.int64).reshape(nb, 8)[:, :6] * 0.01     # us
    t -= t[:, 0].min()
    start, end = t[:, 0], t[:, 5]
    print(f"batch {r}: resampled last step {out[-1]['resampled']}; span {end.max():.2f} us; "
          f"start p0/50/90/100 {np.percentile(start, [0, 50, 90, 100]).round(2)}")
    hist, edges = np.histogram(start, bins=12)
    print("  start histogram:", " ".join(f"{e:.1f}:{h}" for e, h in zip(edges[:-1], hist)))
    late = start > 0.5 * end.max() * 0.5
    for label, sel in (("early", ~late), ("late", late)):
        if not sel.any():
            continue
        d = np.diff(t[sel], axis=1)
        med = np.median(d, axis=0)
        p90 = np.percentile(d, 90, axis=0)
        print(f"  {label:5s} blocks {sel.sum():5d}: " + "  ".join(
            f"{n} {m:5.2f}/{q:5.2f}" for n, m, q in zip(names, med, p90)) +
            f"  | end p50/max {np.median(end[sel]):.2f}/{end[sel].max():.2f}")
