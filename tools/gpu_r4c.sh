#!/bin/bash
# round 4: fused-kernel phase timeline (probe build), MT stream parity with the
# 16-byte candidate loads, then a bench line with the alternate modes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4c}
mkdir -p $out
timeout -k 10 150 python tools/fused_probe.py > $out/fprobe.txt 2>&1
rc=$?; cat $out/fprobe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_rng.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/rng.log 2>&1
rc=$?; echo "pytest rng rc=$rc"; tail -3 $out/rng.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $out/bench20.json 2> $out/bench20.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] && python tools/bench_brief.py $out/bench20.json; exit $rc
