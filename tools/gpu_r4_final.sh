#!/bin/bash
# round 4 evidence, part 1: smoke, every GPU test, the default bench line and
# rocprofv3 kernel statistics of the bench (the PMC passes are part 2:
# tools/gpu_pmc.sh r4 -- a separate call, they take ~10 minutes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4final}
mkdir -p $out
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench.err; exit $rc; }
python tools/bench_brief.py $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o prof -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/prof.err; exit $rc; }
python tools/trace_summary.py $out/prof/prof_kernel_trace.csv > $out/trace_summary.txt; head -14 $out/trace_summary.txt
