"""Graph C5 cond estimate vs its stopping tolerance (development probe): per
Gauss-Newton update the wall time, the estimate's iterations per side, its
lambda_min / lambda_max and device time, for a few cond_tol values."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
from slamhip.graph import DeviceGraph, circle_graph  # noqa: E402

init, truth, edges = circle_graph(50000, n_landmarks=64, seed=0, odom_noise=0.002)
tols = [float(t) for t in sys.argv[1:]] or [1e-5, 3e-5, 1e-4]
for tol in tols:
    dev = DeviceGraph(solver="pcg", pcg_tol=1e-10, cond_tol=tol)
    dev.set_poses(init)
    dev.set_edges(edges)
    for u in range(5):
        t0 = time.perf_counter()
        st = dev.update()
        el = time.perf_counter() - t0
        ci, tm = dev.cond_info(), dev.timing()
        print(f"tol {tol:.0e} update {u}: {el * 1e3:7.3f} ms  solve {tm['solve_ms']:.3f}  "
              f"pcg {tm['pcg_iterations']}  est iters {ci['iterations']} "
              f"(min {ci['iterations_min']}, max {ci['iterations_max']})  "
              f"lmin {ci['lambda_min']:.9e}  lmax {ci['lambda_max']:.9e}  est {ci['ms']:.3f} ms  "
              f"calc {int(st[0])}", flush=True)
    dev.close()
