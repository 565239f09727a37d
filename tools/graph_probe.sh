#!/bin/bash
# PCG kernel times (rocprofv3) of the C5 row for the default library and each
# variant in $LIBS (tools/build_variant.sh NAME "-D..." builds one).  The
# round-1 probes (redundant fold removed, z gathered at s % 50000) were
# temporary -D switches in graph_kernels.inl; DESIGN.md section 8 has their numbers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gprobe}
mkdir -p "$OUT"
for L in hip ${LIBS:-}; do
  SLAM_HIP_LIB=slam-robot_simu_amd/slamhip/libslam_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$L" -o run -- python tools/sec_bench.py graph > "$OUT/$L.log" 2>&1 || exit $?
  echo "$L"
  python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pcg' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'])
" "$OUT/$L/run_kernel_stats.csv"
done
