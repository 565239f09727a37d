#!/bin/bash
# round 4: full GPU suite after the run() setup / export changes, the
# per-call overhead, table-staging A/B, bench at 20 and 50 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4e}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/run_overhead.py > $out/overhead.txt 2>&1
rc=$?; tail -3 $out/overhead.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in libslam_hip.so libslam_tablate.so; do
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/variant_bench.py >> $out/variants.txt 2>&1
    rc=$?; echo "$(tail -1 $out/variants.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20.json 2> $out/bench20.err && timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50.json 2> $out/bench50.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] && python tools/bench_brief.py $out/bench20.json $out/bench50.json; exit $rc
