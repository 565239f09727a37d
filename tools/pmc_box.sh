#!/bin/bash
# PMC passes + their summary on the GPU box (development tool): the raw
# per-dispatch CSVs exceed what gpurun copies back, so only the summaries
# (profiles/<tag>_pmc.json, profiles/pmc_traffic.json) return, under gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r6pmc}
bash tools/pmc.sh || exit 1
python tools/pmc_parse.py gpurun_out/$TAG ${PTAG:-r6} > gpurun_out/$TAG/parse.txt 2>&1 || { tail -5 gpurun_out/$TAG/parse.txt; exit 1; }
cp profiles/${PTAG:-r6}_pmc.json profiles/pmc_traffic.json gpurun_out/$TAG/
rm -rf gpurun_out/$TAG/p[0-9]*/
head -40 gpurun_out/$TAG/parse.txt
