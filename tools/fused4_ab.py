"""Interleaved A/B of the fused-kernel forms on the C2 step (development tool):
one-round (four particles per lane) against two particles per lane, both in
one process through slam_pf_set_fused_one_round, each measured as bench.py
does (graphs captured, settle, warm-up, timed batch, event pass).

    python tools/fused4_ab.py [rounds] [likelihood]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402
from slamhip.pf import DeviceParticleFilter  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
lik = sys.argv[2] if len(sys.argv) > 2 else "logsum"
settle, warm, steps = 4 * bench.SETTLE_BATCH, 5, 50
total = settle + warm + 2 * steps
lm, zs, (vel, omega, dt) = bench.simulate_world(total)
ctl = np.tile([vel, omega], (total, 1))


def one(flag):
    pf = DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity", likelihood=lik, seed=3)
    try:
        pf.set_fused_one_round(flag)
        pf.load_observations(zs)
        pf.prepare_graphs()
        s0 = bench.settle(pf.run, ctl, settle)
        pf.run(s0, ctl[s0:s0 + warm], want_results=False)
        pf.run(s0 + warm, ctl[s0 + warm:s0 + warm + 1], want_results=False)
        t0 = time.perf_counter()
        pf.run(s0 + warm + 1, ctl[s0 + warm + 1:s0 + warm + 1 + steps])
        el = time.perf_counter() - t0
        pf.enable_timing(True)
        a = s0 + warm + 1 + steps
        pf.run(a, ctl[a:a + steps - 1])
        f, r, s = pf.timing(0), pf.timing(1), pf.timing(2)
        pf.enable_timing(False)
        return el / steps * 1e3, f[0] / max(f[1], 1) * 1e3, r[0] / max(r[1], 1) * 1e3, \
            s[0] / max(s[1], 1) * 1e3
    finally:
        pf.close()


for rd in range(rounds):
    for flag in (True, False):
        st, fu, fi, sc = one(flag)
        print(f"round {rd} {'one-round' if flag else 'pair     '} {lik}: step {st:.4f} ms  "
              f"fused {fu:.1f} us  finalize {fi:.1f} us  scan {sc:.1f} us", flush=True)
