#!/bin/bash
# Fused-kernel time and VALU instruction count against the landmark count
# (development tool): NL = 1 isolates the per-particle work (predict, RNG,
# exp, epilogue), the slope the per-update cost.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcnl}
mkdir -p "$OUT"
for v in ${LIBS:-libslam_hip.so}; do
  echo "== $v"
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -k 10 120 python tools/nl_sweep.py || exit $?
  SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v NLS="1 100" timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --output-format csv -d "$OUT/${v%.so}" -o pmc -- python tools/nl_sweep.py > "$OUT/${v%.so}.txt" 2>&1 || exit $?
done
echo done
