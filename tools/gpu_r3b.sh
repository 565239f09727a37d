#!/bin/bash
# round-3 evidence pass: every GPU test (failures reported, not fatal), then the
# default bench line, a rocprofv3 kernel-trace/stats run of the bench and the
# PMC passes of tools/pmc.sh.  Any crash, abort or time limit (rc > 1) ends it.
#   tools/gpu_r3b.sh <tag> [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest "${@:-tests}" -m gpu -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o prof -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/prof.err; exit $rc; }
TAG=${tag}_pmc BENCH_ARGS="--no-secondary" PMC_TIMEOUT=200 tools/pmc.sh
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the driver's own command: default flags (cpu_baseline and secondary rows)
timeout -k 10 600 python bench.py > $out/bench_default.json 2> $out/bench_default.err
rc=$?; echo "default bench rc=$rc"; exit $rc
