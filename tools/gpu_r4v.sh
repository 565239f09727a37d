#!/bin/bash
# round 4: the set_edges spike -- wall times with default and eager code-object
# loading, then a HIP runtime + kernel + copy trace of the probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4v}
mkdir -p $out
echo "== default" > $out/probe.txt
timeout -k 10 120 python -u tools/graph_build_probe.py >> $out/probe.txt 2>&1 || exit 1
echo "== HIP_ENABLE_DEFERRED_LOADING=0" >> $out/probe.txt
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 python -u tools/graph_build_probe.py >> $out/probe.txt 2>&1 || exit 1
cat $out/probe.txt
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $out/rt -o rt -- python -u tools/graph_build_probe.py > $out/rt.txt 2>&1
rc=$?; tail -8 $out/rt.txt; ls $out/rt; exit $rc
