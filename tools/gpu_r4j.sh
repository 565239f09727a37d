#!/bin/bash
# round 4: PF / graph tests after the lazy run results, the spin-then-block
# batch wait and the graph revert; per-call cost with / without the spin and
# under a HIP API trace; bench at 20 and 50 steps twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4j}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_dist.py tests/test_gpu_graph_cond.py tests/test_gpu_rng.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for sp in 1 0 1 0; do
  SLAM_SPIN_WAIT=$sp timeout -k 10 200 python tools/run_overhead.py > $out/ovh_$sp.txt 2>&1 || exit $?
  echo "spin=$sp $(tail -1 $out/ovh_$sp.txt)"
done
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d $out/rt -o rt -- python tools/run_overhead.py > $out/rt.txt 2>&1
echo "runtime trace rc=$?"
for r in 1 2; do
  timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20_$r.json 2> $out/bench20_$r.err || exit $?
  timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50_$r.json 2> $out/bench50_$r.err || exit $?
done
python tools/bench_brief.py $out/bench20_1.json $out/bench50_1.json $out/bench20_2.json $out/bench50_2.json
