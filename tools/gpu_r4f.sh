#!/bin/bash
# round 4: first-batch penalty (with / without priming), persistent fused grid
# A/B (same library, SLAM_FUSED_GRID) against the previous build, fused timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4f}
mkdir -p $out
L=$PWD/slam-robot_simu_amd/slamhip
for p in 0 400 0 400; do
  PRIME=$p timeout -k 10 120 python tools/first_run_probe.py >> $out/first.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $out/first.txt; exit $rc; }
done
cat $out/first.txt
for r in 1 2 3; do
  SLAM_HIP_LIB=$L/libslam_hip.so timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1 || exit $?
  echo "$(tail -1 $out/variants.txt)"
  SLAM_HIP_LIB=$L/libslam_loop.so timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1 || exit $?
  echo "persist: $(tail -1 $out/variants.txt)"
  SLAM_FUSED_GRID=full SLAM_HIP_LIB=$L/libslam_loopnl.so timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1 || exit $?
  echo "full: $(tail -1 $out/variants.txt)"
  SLAM_HIP_LIB=$L/libslam_loopnl.so timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1 || exit $?
  echo "persist: $(tail -1 $out/variants.txt)"
done
SLAM_HIP_LIB=$L/libslam_fprobeloopnl.so timeout -k 10 150 python tools/fused_probe.py > $out/fprobe.txt 2>&1
rc=$?; tail -12 $out/fprobe.txt; exit $rc
