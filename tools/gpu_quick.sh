# selected GPU test files, then the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 600 python -u -m pytest "$@" -x -v -rA -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E  " $out/pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json
exit $rc
