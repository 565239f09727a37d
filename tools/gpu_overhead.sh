#!/bin/bash
# round 4: run() per-call overhead probe, plain and under a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-ovh}
mkdir -p $out
timeout -k 10 200 python tools/run_overhead.py > $out/overhead.txt 2>&1
rc=$?; cat $out/overhead.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o ovh -- python tools/run_overhead.py > $out/prof.txt 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
