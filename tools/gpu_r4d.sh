#!/bin/bash
# round 4: run() per-call overhead, the fused-kernel timeline, MT parity, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_overhead.sh ovh || exit $?
bash tools/gpu_r4c.sh r4c
