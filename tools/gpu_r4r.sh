#!/bin/bash
# round 4: graph C5 with the PCG and cond-estimate launches interleaved at
# submission (libslam_hip) vs the PCG batch first (libslam_grold): graph
# parity tests, then tools/graph_cond_tol.py at the default tolerance
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4r}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_cond.py tests/test_gpu_graph.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in libslam_hip.so libslam_grold.so; do
    echo "== $v" >> $out/ab.txt
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 200 python -u tools/graph_cond_tol.py 1e-5 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
cat $out/ab.txt
