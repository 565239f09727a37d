"""One line per bench JSON: the headline and the step breakdown."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    b = d["breakdown_ms_per_step"]
    am = d.get("alt_modes", {})
    print(f, f"{d['value']:.4e}", f"ms/step {d['ms_per_step']:.4f}", f"fused {b['fused']:.4f}",
          f"reduce {b['reduce']:.4f}", f"resample {b['resample']:.4f}", "capture", d.get("graph_capture_ms"),
          "sharded1", round(d.get("sharded1", {}).get("over_single", 0), 3),
          "product", round(am.get("product", {}).get("fused_avg_ms", 0), 4),
          "numpy", round(am.get("numpy_stream", {}).get("ms_per_step", 0), 4),
          "strong", round(d.get("strong_single", {}).get("ms_per_step", 0), 4),
          "resamples", d.get("resample_steps"))
