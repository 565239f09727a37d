cd $GRAFT_REPO_ROOT
for v in hip inl noslow hip; do
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/libslam_$v.so timeout -k 10 120 python tools/variant_bench.py || exit 1
done
mkdir -p gpurun_out/r2d
timeout -k 10 900 python -m pytest tests/test_gpu_pf.py tests/test_gpu_c2.py tests/test_gpu_configs.py -q -rA -s --timeout 400 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "max relative|passed|failed|^E  " gpurun_out/r2d/pytest.log | head -40
