#!/bin/bash
# round-3: A/B of the working tree against HEAD (libslam_base.so), then the PF tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r3i}; out=gpurun_out/$tag; mkdir -p $out
tools/ab.sh $tag 3 libslam_base.so libslam_hip.so || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_dist.py tests/test_gpu_ess_near.py ${EXTRA_TESTS} -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; exit $rc
