#!/bin/bash
# round 4: the cond estimate's stall window (SLAM_GRAPH_COND_WIN) -- the cond
# accuracy tests at window 8, then iterations / values / time per update for
# (window, tol) = (16, 1e-5), (8, 5e-6), (8, 1e-5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4t}
mkdir -p $out
SLAM_GRAPH_COND_WIN=8 timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_cond.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest_w8.log 2>&1
echo "pytest (window 8) rc=$?"; tail -3 $out/pytest_w8.log
for r in 1 2; do
  echo "== window 16" >> $out/ab.txt
  timeout -k 10 200 python -u tools/graph_cond_tol.py 1e-5 >> $out/ab.txt 2>&1 || exit 1
  echo "== window 8" >> $out/ab.txt
  SLAM_GRAPH_COND_WIN=8 timeout -k 10 200 python -u tools/graph_cond_tol.py 5e-6 1e-5 >> $out/ab.txt 2>&1 || exit 1
done
cat $out/ab.txt
