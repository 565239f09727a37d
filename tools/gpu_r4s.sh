#!/bin/bash
# round 4: graph C5 cond estimate with the fold in the SpMV launch's last
# workgroup (two launches per iteration, default) vs the separate fold launch
# (SLAM_GRAPH_COND_MERGED=0): graph parity tests, then tools/graph_cond_tol.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4s}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_cond.py tests/test_gpu_graph.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for m in 1 0; do
    echo "== merged=$m" >> $out/ab.txt
    SLAM_GRAPH_COND_MERGED=$m timeout -k 10 200 python -u tools/graph_cond_tol.py 1e-5 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
SLAM_GRAPH_COND_MERGED=1 timeout -k 10 300 python -u tools/graph_c5_ab.py >> $out/ab.txt 2>&1
cat $out/ab.txt
