#!/bin/bash
# round-3 quick pass: selected GPU tests, the instruction-rate probe, the
# default bench line.  tools/gpu_quick3.sh <tag> <pytest args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
if [ -x tools/inst_rate ] && [ ! -f $out/inst_rate.txt ] && [ -n "$INST" ]; then
  timeout -k 10 120 tools/inst_rate > $out/inst_rate.txt 2>&1; rc=$?; cat $out/inst_rate.txt; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench.err; exit $rc; }
python -c "import json; d=json.load(open('$out/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'fused', d['roofline']['avg_launch_ms'], 'product', d['alt_modes']['product']['fused_avg_ms'])"
