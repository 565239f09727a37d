#!/bin/bash
# nl_sweep.py over several in-tree library builds (development tool).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${LIBS:-libslam_hip.so}; do
  echo "== $v"
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/nl_sweep.py || exit $?
done
