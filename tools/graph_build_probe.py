"""Wall time of DeviceGraph.set_edges at C5 (bench_graph's structure_build_ms),
repeated, for a rocprofv3 kernel + memory-copy trace of the same calls."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-robot_simu_amd"))
from slamhip.graph import DeviceGraph, circle_graph  # noqa: E402

init, truth, edges = circle_graph(50000, n_landmarks=64, seed=0, odom_noise=0.002)
dev = DeviceGraph(solver="pcg", pcg_tol=1e-10)
dev.set_poses(init)
for k in range(int(os.environ.get("PROBE_CALLS", "6"))):
    t0 = time.perf_counter()
    dev.set_edges(edges)
    el = (time.perf_counter() - t0) * 1e3
    if not os.environ.get("PROBE_QUIET") or el > 4.0:
        print(f"set_edges {k}: {el:.3f} ms", flush=True)
dev.close()
