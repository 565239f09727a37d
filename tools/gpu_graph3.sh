#!/bin/bash
# round-3: graph tests and the C5 row (with / without the cond estimate), plus a trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-g3}
mkdir -p $out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_cond.py tests/test_gpu_graph.py tests/test_gpu_configs.py -m gpu -v -rA --timeout 300 --timeout-method thread -k "cond or graph or c5" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/sec_bench.py graph > $out/sec_noprof.json 2> $out/sec_noprof.err
rc=$?; echo "sec rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/sec_noprof.err; exit $rc; }
python -c "import json; d=json.loads(open('$out/sec_noprof.json').read().split(' ',1)[1])['graph_c5']; print('NOPROF', {k: d[k] for k in ('ms_per_iteration','ms_per_iteration_without_cond','cond')}, d['breakdown_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o g -- python tools/sec_bench.py graph > $out/sec.json 2> $out/sec.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/sec.err; exit $rc; }
python tools/trace_summary.py $out/prof/g_kernel_trace.csv | grep -E "cond|pcg" 
python -c "import json; d=json.loads(open('$out/sec.json').read().split(' ',1)[1])['graph_c5']; print({k: d[k] for k in ('ms_per_iteration','ms_per_iteration_without_cond','cond')}); print(d['cond_estimate']); print(d['cond_estimate_first_update'])"
