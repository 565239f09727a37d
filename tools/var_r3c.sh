#!/bin/bash
# round-3: inline vs pre-drawn motion noise (SLAM_PF_PREDRAW), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var3c
for r in 1 2; do
  for pd in 0 1; do
    SLAM_PF_PREDRAW=$pd timeout -k 10 120 python tools/variant_bench.py >> gpurun_out/var3c/variants.txt 2>&1
    rc=$?; echo "predraw=$pd $(tail -1 gpurun_out/var3c/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
