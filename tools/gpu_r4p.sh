#!/bin/bash
# round 4: product factor's exp(-q/2) without the multiply by 1/2 (exp_nhalf) --
# product parity tests, then an interleaved A/B against the previous kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4p}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_closed_form.py -m gpu -x -q --timeout 300 --timeout-method thread -k "product or exp" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
export VB_LIK=product
bash tools/ab.sh ${1:-r4p} 3 libslam_hip.so libslam_prodnh.so
