#!/bin/bash
# round 4: the particle-filter GPU tests, then a bench line (no secondary rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-pf4}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_rng.py tests/test_gpu_ess_near.py tests/test_gpu_closed_form.py tests/test_gpu_philox.py tests/test_gpu_frontends.py -m gpu -x -v -rA --timeout 300 --timeout-method thread -k "not c4 and not c5" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50.json 2> $out/bench50.err
rc=$?; echo "bench50 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench50.err; exit $rc; }
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20.json 2> $out/bench20.err
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench20.err; exit $rc; }
python tools/bench_brief.py $out/bench50.json $out/bench20.json
