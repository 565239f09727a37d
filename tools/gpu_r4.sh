#!/bin/bash
# round 4: every GPU test, then the driver's bench command and a 50-step line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r4}; shift
out=gpurun_out/$tag
mkdir -p $out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $out/pytest.log | tail -30
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 500 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary > $out/bench20.json 2> $out/bench20.err
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench20.err; exit $rc; }
timeout -k 10 500 python bench.py --warmup 5 --steps 50 --no-cpu-baseline --no-secondary > $out/bench50.json 2> $out/bench50.err
rc=$?; echo "bench50 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench50.err; exit $rc; }
python - $out <<'PY'
import json, sys
for n in ("bench20", "bench50"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    b = d["breakdown_ms_per_step"]
    print(n, f"{d['value']:.3e}", f"ms/step {d['ms_per_step']:.4f}", f"fused {b['fused']:.4f}",
          f"reduce {b['reduce']:.4f}", f"resample {b['resample']:.4f}", "capture", d.get("graph_capture_ms"),
          "sharded1", d.get("sharded1", {}).get("over_single"), "product", d["alt_modes"]["product"]["fused_avg_ms"],
          "numpy", d["alt_modes"]["numpy_stream"]["ms_per_step"])
PY
