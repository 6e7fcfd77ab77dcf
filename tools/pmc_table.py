#!/usr/bin/env python3
"""Per-kernel (name, grid) means of rocprofv3 counter-collection CSVs, one
column per counter, plus derived ratios (tools/pmc_limits.sh).
usage: tools/pmc_table.py <dir-or-csv>... [--match SUBSTR]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name.replace("void ", "")).replace("hpdct::", "")
    return name.replace("unsigned char", "u8").replace("signed char", "i8").replace("true", "T").replace("false", "F")


def load(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        files = [p] if p.endswith(".csv") else glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
        for f in files:
            for r in csv.DictReader(open(f)):
                key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args.remove(match)
    acc = load(args)
    for (k, grid), ctr in sorted(acc.items()):
        if match and match not in k:
            continue
        m = {c: sum(v) / len(v) for c, v in ctr.items()}
        n = len(next(iter(ctr.values())))
        line = f"{k[:60]:60s} grid {grid:9d} n={n:3d} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()))
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_WAIT_INST_ANY", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS"):
                if c in m:
                    line += f" | {c}/wave={m[c] / w:.1f}"
        print(line)


if __name__ == "__main__":
    main()
