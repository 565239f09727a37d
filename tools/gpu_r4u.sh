#!/bin/bash
# round 4: the PMC passes of the fused kernels on the round's final sources
# (tools/pmc.sh), parsed on the box into profiles/r4_pmc.json and
# profiles/pmc_traffic.json; the raw per-dispatch tables are dropped (they
# exceed gpurun_out's 64 MiB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r4 BENCH_ARGS="--no-secondary" PMC_TIMEOUT=200 bash tools/pmc.sh || exit $?
python tools/pmc_parse.py gpurun_out/r4 r4 > gpurun_out/r4_pmc_parse.txt 2>&1 || { tail -5 gpurun_out/r4_pmc_parse.txt; exit 1; }
mkdir -p gpurun_out/r4_profiles && cp profiles/r4_pmc.json profiles/pmc_traffic.json gpurun_out/r4_profiles/
for d in gpurun_out/r4/p*/; do rm -rf "$d"; done
du -sh gpurun_out
head -30 gpurun_out/r4_pmc_parse.txt
