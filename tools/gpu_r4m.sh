#!/bin/bash
# round 4: MT ring refill with two segments per round workgroup -- the device
# stream's bit-exact tests, then the NumPy-stream step A/B against one segment
# per workgroup (libslam_seg1), and a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4m}
mkdir -p $out
L=$PWD/slam-robot_simu_amd/slamhip
timeout -k 10 400 python -u -m pytest tests/test_gpu_rng.py tests/test_gpu_c2.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in libslam_hip.so libslam_seg1.so; do
    SLAM_HIP_LIB=$L/$v timeout -k 10 200 python tools/ns_ab.py >> $out/ab.txt 2>&1 || { tail -3 $out/ab.txt; exit 1; }
    tail -1 $out/ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o ns -- python tools/ns_ab.py > $out/prof.txt 2>&1
echo "prof rc=$?"
