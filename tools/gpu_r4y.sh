#!/bin/bash
# round 4: set_edges spikes -- 300 calls each, pinned read-back of the counts and
# times (libslam_hip) vs the pageable read-back (libslam_sedold), twice
# interleaved; only calls over 4 ms are printed; graph tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4y}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_graph_cond.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in libslam_hip.so libslam_sedold.so; do
    echo "== $v" >> $out/spikes.txt
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v PROBE_CALLS=300 PROBE_QUIET=1 timeout -k 10 200 python -u tools/graph_build_probe.py >> $out/spikes.txt 2>&1 || exit 1
  done
done
cat $out/spikes.txt
