"""Per-kernel duration distribution of a rocprofv3 kernel trace (csv), one
line per (kernel, grid size): the bench's N = 1 command launches the fused
kernel at 2^20 particles (the headline) and at 2^23 (strong_single), whose
launches rocprofv3's --stats summary averages together.

    python tools/trace_summary.py gpurun_out/<tag>/prof/prof_kernel_trace.csv [out.csv]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("slam::", "")
    g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    d[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
out = []
for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    avg = sum(v) / len(v)
    out.append((k, g, len(v), avg, v2[0], v2[len(v) // 2], v2[-1], sum(v)))
    print(f"{k[:45]:45s} grid={g:9d} n={len(v):4d} avg={avg:7.1f} min={v2[0]:7.1f} "
          f"med={v2[len(v) // 2]:7.1f} max={v2[-1]:7.1f} tot={sum(v):9.1f} us")
if len(sys.argv) > 2:
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_size", "calls", "avg_us", "min_us", "median_us", "max_us", "total_us"])
        for rec in out:
            w.writerow([rec[0], rec[1], rec[2]] + [f"{x:.3f}" for x in rec[3:]])
