#!/bin/bash
# round-3: product-mode fused kernel, table exp; default vs no waves-per-EU cap
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var3d
for r in 1 2; do
  for v in libslam_hip.so libslam_pwpe0.so; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v VB_LIK=product timeout -k 10 120 python tools/variant_bench.py >> gpurun_out/var3d/variants.txt 2>&1
    rc=$?; echo "product $(tail -1 gpurun_out/var3d/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
