cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1 BENCH_ARGS="--no-secondary" PMC_TIMEOUT=200 bash tools/pmc.sh && python tools/pmc_parse.py gpurun_out/$1 $1 && cp profiles/$1_pmc.json profiles/pmc_traffic.json gpurun_out/$1/
