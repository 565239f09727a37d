#!/bin/bash
# Interleaved A/B of library variants on the C2 step (development tool):
#   tools/ab.sh TAG ROUNDS LIB... ; VB_LIK=product for the product mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq $rounds); do
  for v in "$@"; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> $out/ab.txt 2>&1
    rc=$?; echo "$(tail -1 $out/ab.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
