#!/bin/bash
# round-3: MT finish step inside the observation kernel -- stream tests, numpy_stream A/B vs HEAD,
# then the default bench line (with the current PMC traffic)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r3o}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rng.py tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_dist.py tests/test_gpu_philox.py -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; [ $rc -le 1 ] || exit $rc
tools/ab.sh $tag 3 libslam_base.so libslam_hip.so || exit $?
for r in 1 2; do for v in libslam_base.so libslam_hip.so; do
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-secondary > $out/b_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$out/b_$v.json')); print('$v', d['ms_per_step'], 'numpy_stream', d['alt_modes']['numpy_stream']['ms_per_step'])"
done; done
timeout -k 10 600 python bench.py > $out/bench_default.json 2> $out/bench_default.err
