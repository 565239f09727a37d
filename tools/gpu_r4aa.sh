#!/bin/bash
# round 4: step graphs of up to 16 steps (default) vs up to 8
# (SLAM_PF_GRAPH_LEVELS=4): PF run tests, then 20- and 50-step lines twice,
# interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4aa}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_ess_near.py tests/test_gpu_bench.py tests/test_gpu_configs.py tests/test_gpu_rng.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lv in 5 4; do
    for k in 20 50; do
      SLAM_PF_GRAPH_LEVELS=$lv timeout -k 10 300 python bench.py --warmup 5 --steps $k --no-secondary --no-cpu-baseline > $out/b${lv}_${k}_$r.json 2> $out/b${lv}_${k}_$r.err || { tail -5 $out/b${lv}_${k}_$r.err; exit 1; }
      echo "levels $lv: $(python tools/bench_brief.py $out/b${lv}_${k}_$r.json)"
    done
  done
done
