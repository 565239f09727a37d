#!/bin/bash
# replay var_r3e.sh's test order in one process
# (philox -> pf -> dist -> c2 -> configs) to reproduce the C2 lockstep cov miss.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-repro}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_philox.py tests/test_gpu_pf.py tests/test_gpu_dist.py tests/test_gpu_c2.py tests/test_gpu_configs.py -m gpu -v -rA --timeout 300 --timeout-method thread -k "not c4 and not c5" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -40
exit $rc
