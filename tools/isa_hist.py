#!/usr/bin/env python
"""Static instruction histogram of one kernel in a hipcc -S dump (device ISA).

    python tools/isa_hist.py /tmp/isa/pf_api.s 'pf_fused_kernelILi1ELi1ELb0ELb1E'

Prints the kernel's register/scratch metadata and its instruction mix by class
(static counts: loop bodies count once; use the PMC SQ_INSTS_* for dynamic).
"""
import re
import sys
from collections import Counter


def kernel_lines(path, pat):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + pat + r"\S*:", l):
            start = i
        elif start is not None and (l.startswith(".Lfunc_end") or l.startswith("\t.size")):
            return lines[start:i], lines[i:i + 200]
    raise SystemExit("kernel not found")


def main():
    path, pat = sys.argv[1], sys.argv[2]
    body, tail = kernel_lines(path, pat)
    ops = Counter()
    for l in body:
        l = l.strip()
        if not l or l.startswith((";", ".", "_")) or l.endswith(":"):
            continue
        ops[l.split()[0]] += 1
    cls = Counter()
    for op, c in ops.items():
        if op.startswith("v_") and "f64" in op:
            k = "valu_f64"
        elif op.startswith(("v_mul_hi", "v_mul_lo", "v_mad_u64", "v_mad_i64", "v_mul_u32")):
            k = "valu_imul"
        elif op.startswith("v_"):
            k = "valu_other"
        elif op.startswith("s_"):
            k = "salu/smem"
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            k = "vmem"
        elif op.startswith("ds_"):
            k = "lds"
        else:
            k = "other"
        cls[k] += c
    print("classes:", dict(cls))
    for op, c in ops.most_common(60):
        print(f"{c:6d} {op}")
    for l in tail:
        if any(k in l for k in ("vgpr_count", "sgpr_count", "NumVgprs", "ScratchSize", "Occupancy",
                                 "private_segment_fixed_size", "agpr_count", "NumVGPRsForWavesPerEU")):
            print(l.strip())


if __name__ == "__main__":
    main()
