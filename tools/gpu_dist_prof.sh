# dist tests, then the sharded bench under rocprofv3 (kernel trace + stats)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r2h}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v -rA -s --timeout 200 --timeout-method thread > $out/pytest_dist.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E  " $out/pytest_dist.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --mode sharded --steps 20 --warmup 3 --no-secondary --no-cpu-baseline > $out/bench.json 2> $out/prof.err
rc=$?; echo "rocprof rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_default.json 2> $out/bench_default.err
rc=$?; echo "bench rc=$rc"; cat $out/bench_default.json
exit $rc
