"""Secondary-row timing (development tool): runs bench.py's EKF batch, EKF-SLAM
C4 and graph C5 rows alone through the library named by SLAM_HIP_LIB."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))
import bench  # noqa: E402

which = sys.argv[1:] or ["ekfslam"]
out = {}
if "ekf" in which:
    out["ekf_batch"] = bench.bench_ekf_batch()
if "ekfslam" in which:
    out["ekfslam_c4"] = bench.bench_ekfslam()
if "graph" in which:
    out["graph_c5"] = bench.bench_graph()
print(os.environ.get("SLAM_HIP_LIB", "default"), json.dumps(out))
