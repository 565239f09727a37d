#!/bin/bash
# VALU/SALU/wave counters of the PF kernels for several in-tree library builds
# (development tool; one counter group per pass, no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcvar
mkdir -p "$OUT"
for v in ${LIBS:-libslam_hip.so}; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    tag=${v%.so}_$(echo $grp | cut -c1-12 | tr ' ' _)
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$tag" -o pmc -- python tools/variant_bench.py > "$OUT/$tag.txt" 2>&1
    rc=$?; echo "$tag rc=$rc"
    if [ $rc != 0 ]; then tail -5 "$OUT/$tag.txt"; exit $rc; fi
  done
done
echo done
