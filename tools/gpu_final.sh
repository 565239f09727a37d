#!/bin/bash
# end of round 3: A/B of the working tree against HEAD (libslam_base.so), then the
# full evidence pass (every GPU test, bench, rocprof, PMC, default bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r3q}
tools/ab.sh $tag 3 libslam_base.so libslam_hip.so || exit $?
tools/gpu_r3b.sh $tag tests
