#!/bin/bash
# round 4: the correlated-R likelihood test (both modes), then the set_edges
# spike investigation (tools/gpu_r4v.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4w}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pf.py -m gpu -x -v --timeout 200 --timeout-method thread -k "correlated or likelihood_stage" -s > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "correlated|likelihood [abc]|passed|failed" $out/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4v.sh ${1:-r4w}
