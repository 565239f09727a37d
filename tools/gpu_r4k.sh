#!/bin/bash
# round 4: NumPy-stream step with the observation on a side graph branch --
# the device-stream parity tests, then bench lines with the branch on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4k}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rng.py tests/test_gpu_pf.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    SLAM_MT_FORK=$f timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench_f${f}_$r.json 2> $out/bench_f${f}_$r.err || exit $?
    echo "fork=$f $(python tools/bench_brief.py $out/bench_f${f}_$r.json)"
  done
done
for r in 1 2; do
  timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50_$r.json 2> $out/bench50_$r.err || exit $?
  echo "50 steps: $(python tools/bench_brief.py $out/bench50_$r.json)"
done
