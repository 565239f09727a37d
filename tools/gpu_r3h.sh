#!/bin/bash
# round-3: DPP-epilogue A/B + PF tests, then the MT round size (requests per round) A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r3h}; mkdir -p $out
tools/ab.sh ${1:-r3h} 3 libslam_base.so libslam_hip.so || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_dist.py tests/test_gpu_ess_near.py tests/test_gpu_rng.py -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for ra in 16 32; do
    SLAM_MT_ROUNDS_AHEAD=$ra timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-secondary > $out/bench_ra$ra.json 2> $out/bench_ra$ra.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $out/bench_ra$ra.err; exit $rc; }
    python -c "import json; d=json.load(open('$out/bench_ra$ra.json')); print('rounds_ahead $ra numpy_stream', d['alt_modes']['numpy_stream']['ms_per_step'], 'step', d['ms_per_step'], 'sharded1', d['sharded1'])"
  done
done
