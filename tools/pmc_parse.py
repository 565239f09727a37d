#!/usr/bin/env python
"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh per kernel.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads
exactly half of a wide coalesced streaming read on gfx950, so it is doubled;
WRITE_SIZE (KB) is taken as is.  Writes profiles/<tag>_pmc.json and, for the
bench, profiles/pmc_traffic.json with the fused kernel's per-launch traffic.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(dirpath):
    """Counters per (kernel, grid size): one kernel launched at several sizes
    (the bench's 2^20 line and its 2^23 strong-scaling reference) is kept
    apart, the 2^20 grid under the plain name, others as 'name @grid G'."""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(collections.Counter)
    rows = []
    for f in glob.glob(os.path.join(dirpath, "p*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            rows.append(r)
            grids[r["Kernel_Name"]][int(r["Grid_Size"])] += 1
    for r in rows:
        name, g = r["Kernel_Name"], int(r["Grid_Size"])
        if len(grids[name]) > 1 and g != FUSED_GRID:
            name = f"{name} @grid {g}"
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        per[name]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return per


FUSED_GRID = (1 << 20) // 2          # the bench's fused grid: 2^20 particles, two per lane


def short(name):
    n = name.replace("slam::", "").replace("void ", "")
    g = n.split(" @grid ")
    return n.split("(")[0] + (f" @grid {g[1]}" if len(g) > 1 else "")


def main(src, tag):
    per = load(src)
    out = {}
    for name, cs in per.items():
        if "rocclr" in name:
            continue
        d = {k: sum(v) / len(v) for k, v in cs.items()}
        rec = {"launch_records": len(cs.get("FETCH_SIZE", [])), "avg_dur_us_profiled": d["_dur_ns"] / 1e3}
        if "FETCH_SIZE" in d:
            rec["hbm_read_bytes"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            rec["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        for k in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                  "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "GRBM_GUI_ACTIVE", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                  "SQ_INSTS_VALU_TRANS_F64"):
            if k in d:
                rec[k] = d[k]
        f64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
               "SQ_INSTS_VALU_TRANS_F64")
        if all(k in d for k in f64):
            # executed fp64 flops per launch: 64 lanes x (add + mul + trans + 2 fma)
            rec["fp64_flops"] = 64 * (d[f64[0]] + d[f64[1]] + d[f64[3]] + 2 * d[f64[2]])
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            rec["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        out[short(name)] = rec
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/{tag}_pmc.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    def summary(key):
        v = out[key]
        rec = {k: v[k] for k in ("fp64_flops", "SQ_INSTS_VALU", "SQ_WAVES", "avg_dur_us_profiled",
                                 "valu_insts_per_wave", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                                 "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                 "GRBM_GUI_ACTIVE") if k in v}
        if "hbm_read_bytes" in v and "hbm_write_bytes" in v:
            rec["hbm_bytes"] = v["hbm_read_bytes"] + v["hbm_write_bytes"]
        return rec

    key = "pf_fused_kernel<1, 1, false, true>"       # the bench's kernel (velocity, log-sum)
    if key in out and "hbm_read_bytes" in out[key] and "hbm_write_bytes" in out[key]:
        main_rec = summary(key)
        kernels = {}
        pkey = "pf_fused_kernel<1, 0, false, true>"  # the reference-literal product mode
        if pkey in out:
            kernels["product"] = summary(pkey)
        sys.path.insert(0, os.getcwd())
        from bench import pf_sources_sha
        with open("profiles/pmc_traffic.json", "w") as f:
            json.dump({"source": f"profiles/{tag}_pmc.json", "kernel": key,
                       "fused_kernel_hbm_bytes_per_launch": main_rec.get("hbm_bytes"),
                       "sources_sha": pf_sources_sha(),
                       "fused_kernel": main_rec, "kernels": kernels,
                       "note": "FETCH_SIZE x2 (gfx950 half-count) + WRITE_SIZE, KB -> B, mean over "
                               "launches; fp64_flops = 64 x (ADD + MUL + TRANS + 2 FMA)_F64"},
                      f, indent=1)
    for k, v in sorted(out.items()):
        print(f"{k:45s} rd {v.get('hbm_read_bytes', 0)/1e6:8.2f} MB  wr {v.get('hbm_write_bytes', 0)/1e6:7.2f} MB"
              f"  valu/wave {v.get('valu_insts_per_wave', 0):8.1f}  waves {v.get('SQ_WAVES', 0):8.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r1")
