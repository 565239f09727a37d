"""Per-launch VALU counts of the fused kernel from tools/pmc_nl.sh output, split
by landmark count (dispatch order: the NL=1 run first, then NL=100)."""
import csv
import glob
import sys
from collections import defaultdict

for d in sorted(glob.glob(sys.argv[1] + "/*/pmc_counter_collection.csv")):
    rows = defaultdict(dict)
    for r in csv.DictReader(open(d)):
        if "pf_fused_kernel" not in r["Kernel_Name"]:
            continue
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(rows)
    half = len(ids) // 2
    print(d)
    for tag, sel in (("NL=1", ids[:half]), ("NL=100", ids[half:])):
        agg = defaultdict(float)
        for i in sel:
            for k, v in rows[i].items():
                agg[k] += v / len(sel)
        w = agg["SQ_WAVES"]
        print("  %-7s waves %6d  " % (tag, w) + "  ".join("%s %.0f" % (k.replace("SQ_INSTS_", ""), v / w)
                                                       for k, v in sorted(agg.items()) if k != "SQ_WAVES"))
