"""Graph C5 Gauss-Newton iteration with the gate's cond estimate (development
probe): bench.bench_graph's numbers, one line per run (round 4: the label's
SLAM_GRAPH_FUSED selected a fused-launch variant that was measured and not kept)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402

r = bench.bench_graph()
ce = r["cond_estimate"]
print(f"fused={os.environ.get('SLAM_GRAPH_FUSED', '1')}: {r['ms_per_iteration']:.3f} ms/iter  "
      f"without cond {r['ms_per_iteration_without_cond']:.3f}  solve {r['breakdown_ms']['solve_ms']:.3f}  "
      f"pcg iters {r['breakdown_ms']['pcg_iterations']}  cond {r['cond']:.6e} iters {ce['iterations']} "
      f"status {ce['status']}  first-update iters {r['cond_estimate_first_update']['iterations']}")
