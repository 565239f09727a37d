#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof summary.
# Stops at the first crash-like exit (fault/abort/segv/timeout); plain test
# failures (pytest exit 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  if crash $rc; then echo "stopping after crash-like exit $rc"; exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-50} --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
  if [ $rc != 0 ]; then exit $rc; fi
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"; find "$OUT/prof" -name "*stats*" | head
  if [ $rc != 0 ]; then tail -20 "$OUT/prof.err"; exit $rc; fi
fi
echo done
