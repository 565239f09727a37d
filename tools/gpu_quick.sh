#!/bin/bash
# Development loop on the GPU box: parity tests, then the landmark sweep with
# the fused kernel's VALU counts (tools/pmc_nl.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
if [ $rc != 0 ]; then exit $rc; fi
TAG=${TAG:-quick}/nl bash tools/pmc_nl.sh
