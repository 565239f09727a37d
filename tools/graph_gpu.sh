#!/bin/bash
# Graph-SLAM development loop on the GPU box: graph parity tests, the C5 row,
# and its kernel statistics.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-graph}
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/sec_bench.py graph > "$OUT/sec.json" 2>&1 || exit $?
cat "$OUT/sec.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python tools/sec_bench.py graph > /dev/null 2>&1 || exit $?
python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:48], r['Calls'], r['AverageNs'])
" "$OUT/prof/run_kernel_stats.csv"
