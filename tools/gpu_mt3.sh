#!/bin/bash
# round-3: the device NumPy stream (bit-exact tests) and its bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-mt3}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rng.py tests/test_gpu_pf.py -m gpu -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench.err; exit $rc; }
python -c "import json; d=json.load(open('$out/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'numpy_stream', d['alt_modes']['numpy_stream'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o p -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/trace_summary.py $out/prof/p_kernel_trace.csv | grep -E "mt_|fused|finalize"
for ra in 4 16; do
  SLAM_MT_ROUNDS_AHEAD=$ra timeout -k 10 300 python bench.py --steps 48 --warmup 8 --no-cpu-baseline --no-secondary > $out/bench_ra$ra.json 2> $out/bench_ra$ra.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $out/bench_ra$ra.err; exit $rc; }
  python -c "import json; d=json.load(open('$out/bench_ra$ra.json')); print('rounds_ahead $ra numpy_stream', d['alt_modes']['numpy_stream']['ms_per_step'])"
done
