"""Duration distribution of selected kernels in a rocprofv3 kernel trace
(development tool): per (kernel, grid) the count and quantiles, split into
the launches below and above `--split` x the fastest one (a device-gated
kernel's no-op launches against its working ones).

    python tools/kdist.py prof/bench_kernel_trace.csv scan_lean finalize [--split 3]
"""
import argparse
import collections
import csv

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("kernels", nargs="*", help="substrings of the kernel names to keep (all if none)")
ap.add_argument("--split", type=float, default=3.0)
args = ap.parse_args()

d = collections.defaultdict(list)
for r in csv.DictReader(open(args.trace)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("slam::", "")
    if args.kernels and not any(a in n for a in args.kernels):
        continue
    g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    d[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)


def q(v):
    v = np.asarray(v)
    if not len(v):
        return "-"
    p = np.percentile(v, [10, 50, 90])
    return f"n={len(v):5d} mean={v.mean():8.2f} p10={p[0]:8.2f} p50={p[1]:8.2f} p90={p[2]:8.2f}"


for (k, g), v in sorted(d.items()):
    v = np.asarray(v)
    lo = v[v < args.split * v.min()]
    hi = v[v >= args.split * v.min()]
    print(f"{k} grid={g}\n   low : {q(lo)}\n   high: {q(hi)}")
