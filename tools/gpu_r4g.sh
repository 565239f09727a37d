#!/bin/bash
# round 4: PF GPU tests after the fused-kernel revert, bench at 20 and 50 steps
# (with the settle phase), twice each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4g}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_dist.py tests/test_gpu_closed_form.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20_$r.json 2> $out/bench20_$r.err || exit $?
  timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50_$r.json 2> $out/bench50_$r.err || exit $?
done
python tools/bench_brief.py $out/bench20_1.json $out/bench50_1.json $out/bench20_2.json $out/bench50_2.json
