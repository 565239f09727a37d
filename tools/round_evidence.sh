# smoke, the full bench line, and rocprofv3 kernel stats of the same bench command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r2ev}
mkdir -p $out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/trace_summary.py $out/prof/run_kernel_trace.csv > $out/trace_summary.txt; head -12 $out/trace_summary.txt
