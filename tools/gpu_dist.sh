cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2e
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v -rA -s --timeout 200 --timeout-method thread > gpurun_out/r2e/pytest_dist.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E  " gpurun_out/r2e/pytest_dist.log | head -40
exit $rc
