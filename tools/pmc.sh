#!/bin/bash
# PMC passes (one counter group per pass, never combined with tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
ARGS="--steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- python bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc != 0 ]; then tail -5 "$OUT/p$i.err"; exit $rc; fi
done
echo done
