cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2f
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -x -v -rA --timeout 150 --timeout-method thread > gpurun_out/r2f/pytest_bench.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E  " gpurun_out/r2f/pytest_bench.log | head -30
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r2f/bench.json 2> gpurun_out/r2f/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2f/bench.json; tail -3 gpurun_out/r2f/bench.err
