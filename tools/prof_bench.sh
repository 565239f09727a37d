# bench.py under rocprofv3 kernel trace + stats; per-kernel duration summary
# usage: prof_bench.sh <out tag> [bench args...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --no-secondary --no-cpu-baseline "$@" > $out/bench.json 2> $out/prof.err
rc=$?; echo "rocprof rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
python tools/trace_summary.py $out/prof/run_kernel_trace.csv
