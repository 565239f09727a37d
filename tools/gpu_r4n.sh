#!/bin/bash
# round 4: NumPy-stream step with the ring refilled every 64 requests instead
# of 32 (SLAM_MT_ROUNDS_AHEAD), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4n}
mkdir -p $out
for r in 1 2 3; do
  for a in 32 64; do
    SLAM_MT_ROUNDS_AHEAD=$a timeout -k 10 200 python tools/ns_ab.py > $out/ab_$a.txt 2>&1 || { tail -3 $out/ab_$a.txt; exit 1; }
    echo "ahead=$a $(tail -1 $out/ab_$a.txt)" | tee -a $out/ab.txt
  done
done
