#!/bin/bash
# which earlier test makes C2's lockstep cov differ (run order of var_r3e.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/bis2
run() {  # name lib tests...
  local name=$1 lib=$2; shift 2
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$lib timeout -k 10 400 python -u -m pytest "$@" -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/bis2/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -E '[0-9]+ (passed|failed)' gpurun_out/bis2/$name.log | tail -1)"
  [ $rc -le 1 ]
}
run dist_hip libslam_hip.so tests/test_gpu_dist.py tests/test_gpu_c2.py -k "dist or lockstep" &&
run pf_hip libslam_hip.so tests/test_gpu_pf.py tests/test_gpu_c2.py -k "not dist" &&
run dist_nosss libslam_nosss.so tests/test_gpu_dist.py tests/test_gpu_c2.py -k "dist or lockstep"
