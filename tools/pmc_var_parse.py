#!/usr/bin/env python
"""Per-variant fused-kernel counters from tools/pmc_variants.sh output
(development tool): VALU / SALU / LDS instructions per wave and the wait
fractions of pf_fused_kernel<1, 1, false, true> at the bench's grid."""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcvar"
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(src, "*_SQ_*"))):
    if not os.path.isdir(d):
        continue
    var = os.path.basename(d).split("_SQ_")[0]
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "pmc_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "pf_fused_kernel<1, 1, false, true>" in r["Kernel_Name"] and int(r["Grid_Size"]) == 1 << 19:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        res[var][k] = sum(v) / len(v)
for var, c in res.items():
    w = c.get("SQ_WAVES", 8192.0)
    line = f"{var:18s}"
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
        if k in c:
            line += f" {k[9:]}/wave {c[k] / w:8.1f}"
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        line += "  wait_any %.2f wait_inst %.2f active %.2f" % (
            c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc)
    print(line)
