#!/bin/bash
# Fused-kernel timing of several in-tree library builds (development tool).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-variants}
mkdir -p "$OUT"
for v in ${LIBS:-libslam_hip.so}; do
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> "$OUT/variants.txt" 2>&1
  rc=$?; tail -1 "$OUT/variants.txt"
  if [ $rc != 0 ]; then echo "rc=$rc"; exit $rc; fi
done
