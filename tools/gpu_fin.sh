#!/bin/bash
# finscan check: PF + dist GPU tests, bench, kernel trace of the bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fin}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pf.py tests/test_gpu_dist.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cut -c1-400 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/trace_summary.py "$OUT/prof/run_kernel_trace.csv" > "$OUT/trace_summary.txt"; head -12 "$OUT/trace_summary.txt"
