#!/bin/bash
# round 4: NumPy-stream A/B: emit blocks summing their predecessors' counts
# (up to 4096 blocks) vs one prefix launch (libslam_mtpre); rng tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4l}
mkdir -p $out
L=$PWD/slam-robot_simu_amd/slamhip
timeout -k 10 300 python -u -m pytest tests/test_gpu_rng.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in libslam_hip.so libslam_mtpre.so; do
    SLAM_HIP_LIB=$L/$v timeout -k 10 200 python tools/ns_ab.py >> $out/ab.txt 2>&1 || { tail -3 $out/ab.txt; exit 1; }
    tail -1 $out/ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o ns -- python tools/ns_ab.py > $out/prof.txt 2>&1
echo "prof rc=$?"
