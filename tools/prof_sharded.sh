cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2g
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2g/prof -o run -- python bench.py --mode sharded --steps 20 --warmup 3 --no-secondary --no-cpu-baseline > gpurun_out/r2g/bench.json 2> gpurun_out/r2g/prof.err
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/r2g/bench.json
f=$(find gpurun_out/r2g/prof -name "*kernel_stats.csv" | head -1); echo $f
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1e3:9.1f} us  total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
