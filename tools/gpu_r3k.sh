#!/bin/bash
# round-3: sharded probe, A/B vs HEAD (single step and sharded1), PF / dist / C2 / C3 tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r3k}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python tools/dist_probe.py > $out/probe.txt 2>&1 || exit $?
tail -3 $out/probe.txt
EXTRA_TESTS="tests/test_gpu_configs.py tests/test_gpu_rng.py" tools/gpu_r3i.sh $tag || exit $?
for r in 1 2; do for v in libslam_base.so libslam_hip.so; do
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-secondary > $out/b_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/b_$v.json')); print('$v', d['ms_per_step'], d['breakdown_ms_per_step'], d['sharded1'])"
done; done
