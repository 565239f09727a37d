#!/bin/bash
# round 4: folded step end A/B (fold / standalone step end / fold with plain
# output stores), interleaved, then a kernel trace of the fold build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-var4a}
mkdir -p $out
for r in 1 2; do
  for v in libslam_hip.so libslam_nofold.so libslam_nofold1.so libslam_foldplain.so; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1
    rc=$?; echo "$(tail -1 $out/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o fold -- python tools/variant_bench.py > $out/prof.txt 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
