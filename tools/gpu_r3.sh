#!/bin/bash
# round-3 GPU session helper: selected GPU tests, then the default bench line.
#   tools/gpu_r3.sh <tag> <pytest args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 1000 python -u -m pytest "$@" -x -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json; tail -5 $out/bench.err
exit $rc
