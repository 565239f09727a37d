#!/bin/bash
# round-3: table-driven Box-Muller A/B, then the RNG / PF / sharded tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-var3e}
mkdir -p $out
for r in 1 2; do
  for v in libslam_hip.so libslam_notab.so; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1
    rc=$?; echo "$(tail -1 $out/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_philox.py tests/test_gpu_pf.py tests/test_gpu_dist.py tests/test_gpu_c2.py tests/test_gpu_configs.py -m gpu -v -rA --timeout 300 --timeout-method thread -k "not c4 and not c5" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
exit $rc
