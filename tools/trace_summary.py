"""Per-kernel duration distribution of a rocprofv3 kernel trace (csv)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("slam::", "")
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{k[:45]:45s} n={len(v):4d} min={v2[0]:7.1f} med={v2[len(v) // 2]:7.1f} "
          f"max={v2[-1]:7.1f} tot={sum(v):9.1f} us")
