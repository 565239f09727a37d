#!/bin/bash
# round 4: graph C5 with the cond estimate in the solve's launches -- parity
# tests, then an interleaved A/B against the two-stream form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4h}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_cond.py tests/test_gpu_graph.py tests/test_gpu_configs.py -m gpu -x -q --timeout 400 --timeout-method thread -k "graph or c5 or cond" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    SLAM_GRAPH_FUSED=$f timeout -k 10 200 python tools/graph_c5_ab.py >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
    tail -1 $out/ab.txt
  done
done
