#!/bin/bash
# EKF-SLAM development loop on the GPU box: EKF parity tests, then the C4 row
# for the default library and each variant named in $LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-eks}
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_ekf.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc = 0 ] || exit $rc
for L in hip ${LIBS:-}; do
  SLAM_HIP_LIB=slam-robot_simu_amd/slamhip/libslam_$L.so timeout -k 10 120 python tools/sec_bench.py ekfslam > "$OUT/eks_$L.json" 2>&1 || exit $?
  python3 -c "
import json, sys
t = open(sys.argv[1]).read(); d = json.loads(t[t.index('{'):])['ekfslam_c4']
print(sys.argv[2], d['ms_per_update'], d['last_update_breakdown_ms'], d['roofline']['avg_launch_ms'])" "$OUT/eks_$L.json" $L
done
