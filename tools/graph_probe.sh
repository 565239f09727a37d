cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp; mkdir -p gpurun_out/gprobe
for L in hip nofold nogather; do
  SLAM_HIP_LIB=slam-robot_simu_amd/slamhip/libslam_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprobe/$L -o run -- python tools/sec_bench.py graph > gpurun_out/gprobe/$L.log 2>&1 || exit $?
  echo $L; grep -h "graph_pcg" gpurun_out/gprobe/$L/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-20,90-
done
