#!/bin/bash
# Round-6 full GPU pass: the -m gpu suite, smoke, the default bench line, and a
# rocprofv3 kernel-trace summary of the same bench command (development tool).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv')
python tools/trace_summary.py $f $OUT/kernel_stats_by_grid.csv > $OUT/trace.txt 2>&1
python tools/kdist.py $f scan_lean finalize pf_fused > $OUT/kdist.txt 2>&1
rm -f $f
echo done
