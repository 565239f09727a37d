#!/bin/bash
# round 4, final tree: the driver's 20-step line and the 50-step line, twice
# each, interleaved on one box (no secondary rows, no CPU baseline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r4z}
mkdir -p $out
for r in 1 2; do
  for k in 20 50; do
    timeout -k 10 300 python bench.py --warmup 5 --steps $k --no-secondary --no-cpu-baseline > $out/bench${k}_$r.json 2> $out/bench${k}_$r.err || { tail -5 $out/bench${k}_$r.err; exit 1; }
    python tools/bench_brief.py $out/bench${k}_$r.json
  done
done
