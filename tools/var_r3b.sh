#!/bin/bash
# round-3: graph-branch concurrency probe, then fused/step timing of library variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var3b
timeout -k 10 120 tools/graph_concurrency > gpurun_out/var3b/graph_concurrency.txt 2>&1; rc=$?
cat gpurun_out/var3b/graph_concurrency.txt; [ $rc -eq 0 ] || exit $rc
LIBS="libslam_hip.so libslam_finwpe0.so" TAG=var3b tools/variants_run.sh
