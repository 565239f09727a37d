#!/bin/bash
# round 4: catch a set_edges spike under a kernel + copy trace (40 calls), so
# the slow call's kernels and copies can be compared with a fast call's
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4x}
mkdir -p $out
PROBE_CALLS=40 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/kt -o kt -- python -u tools/graph_build_probe.py > $out/kt.txt 2>&1
rc=$?; grep set_edges $out/kt.txt | sort -t: -k2 -n -r | head -5; ls $out/kt; exit $rc
