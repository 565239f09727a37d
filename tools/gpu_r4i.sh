#!/bin/bash
# round 4: PF / sharded (incl. the collective mode) GPU tests and bench lines at
# 20 and 50 steps, then the graph C5 fused-estimate tests and A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4g.sh r4g || exit $?
bash tools/gpu_r4h.sh r4h || exit $?
out=gpurun_out/r4s
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o s1 -- python tools/sharded1_probe.py > $out/probe.txt 2>&1
rc=$?; echo "sharded1 prof rc=$rc"; grep -E "ms/step" $out/probe.txt
