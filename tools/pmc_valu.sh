#!/bin/bash
# VALU-mix counters of the fused kernel for one or more in-tree library builds
# (development tool; one counter group per pass, no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcvalu}
mkdir -p "$OUT"
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1; echo "list rc=$?"
fi
i=0
for v in ${LIBS:-libslam_hip.so}; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"; do
    i=$((i+1))
    SLAM_HIP_LIB=$PWD/slam-robot_simu_amd/slamhip/$v timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${v%.so}_p$i" -o pmc -- python tools/variant_bench.py > "$OUT/${v%.so}_p$i.txt" 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; tail -1 "$OUT/${v%.so}_p$i.txt"
    if [ $rc != 0 ]; then tail -5 "$OUT/${v%.so}_p$i.txt"; exit $rc; fi
  done
done
echo done
