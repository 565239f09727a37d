"""Interleaved A/B of library variants on the C2 step (development tool): each
variant (an in-tree libslam_<name>.so, tools/build_variant.sh) in its own
process per round, measured as bench.py does -- graphs captured, 124 settle
steps, 5 warm-up, 50 timed steps, then an event pass over 49 more.

    python tools/variant_ab.py ROUNDS LIB [LIB ...]      (LIB: file name under slamhip/)
    VB_LIK=product for the product likelihood; VB_ESS=<threshold> (0: never resample);
    VB_NP=<particles> (default the bench's 2^20)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
    import numpy as np
    import bench
    from slamhip.pf import DeviceParticleFilter
    settle, warm, steps = 4 * bench.SETTLE_BATCH, 5, 50
    total = settle + warm + 2 * steps
    lm, zs, (vel, omega, dt) = bench.simulate_world(total)
    ctl = np.tile([vel, omega], (total, 1))
    kw = {"ess_threshold": float(os.environ["VB_ESS"])} if "VB_ESS" in os.environ else {}
    n = int(os.environ.get("VB_NP", bench.NP_PER_GPU))
    pf = DeviceParticleFilter(n, lm, dt=dt, motion="velocity",
                              likelihood=os.environ.get("VB_LIK", "logsum"), seed=3, **kw)
    pf.load_observations(zs)
    pf.prepare_graphs()
    s0 = bench.settle(pf.run, ctl, settle)
    pf.run(s0, ctl[s0:s0 + warm], want_results=False)
    a = s0 + warm
    t0 = time.perf_counter()
    pf.run(a, ctl[a:a + steps])
    el = time.perf_counter() - t0
    pf.enable_timing(True)
    pf.run(a + steps, ctl[a + steps:a + 2 * steps - 1])
    f, r, s = pf.timing(0), pf.timing(1), pf.timing(2)
    pf.close()
    print(f"{os.path.basename(os.environ.get('SLAM_HIP_LIB', 'default'))}: step {el / steps * 1e3:.4f} ms  "
          f"fused {f[0] / max(f[1], 1) * 1e3:.2f} us  finalize {r[0] / max(r[1], 1) * 1e3:.2f} us  "
          f"scan {s[0] / max(s[1], 1) * 1e3:.2f} us", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        sys.exit(0)
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ, SLAM_HIP_LIB=os.path.join(ROOT, "slam-robot_simu_amd", "slamhip", lib))
            rc = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                                timeout=240).returncode
            if rc:
                sys.exit(rc)
