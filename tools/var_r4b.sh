#!/bin/bash
# round 4: fused-kernel RNG placement A/B (loads first / staggered half / RNG
# first), interleaved on one box, then the PF tests through the stagger build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-var4b}
mkdir -p $out
for r in 1 2 3; do
  for v in libslam_hip.so libslam_stagger.so libslam_rngfirst.so; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1
    rc=$?; echo "$(tail -1 $out/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/libslam_stagger.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_dist.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c4 and not c5" > $out/pytest.log 2>&1
rc=$?; echo "pytest(stagger) rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20.json 2> $out/bench20.err && timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50.json 2> $out/bench50.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] && python tools/bench_brief.py $out/bench20.json $out/bench50.json; exit $rc
