#!/bin/bash
# round 4: product-loop A/B (tools/gpu_r4p.sh), then the graph C5 cond
# estimate's iterations and values against its stopping tolerance
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_r4p.sh ${1:-r4q} || exit $?
timeout -k 10 400 python -u tools/graph_cond_tol.py 1e-5 3e-5 1e-4 > gpurun_out/${1:-r4q}/cond_tol.txt 2>&1
rc=$?; cat gpurun_out/${1:-r4q}/cond_tol.txt | tail -16; exit $rc
