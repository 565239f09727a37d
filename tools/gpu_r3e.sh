#!/bin/bash
# round-3 evidence: every GPU test, the bench line with the secondary rows, and
# a rocprofv3 kernel-trace/stats run of the secondary rows (eks_*, graph_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/secprof -o sec -- python tools/sec_bench.py ekf ekfslam graph > $out/sec.json 2> $out/sec.err
rc=$?; echo "secprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/sec.err; exit $rc; }
