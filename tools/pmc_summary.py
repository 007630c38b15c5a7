#!/usr/bin/env python
"""Summarise rocprofv3 counter_collection.csv files: per kernel (name filter) mean value per counter,
for dispatches with the largest grid (the batch launch)."""
import csv
import sys
from collections import defaultdict


def main(pattern, *paths):
    vals = defaultdict(list)
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        rows = [r for r in rows if pattern in r["Kernel_Name"]]
        if not rows:
            continue
        g = max(int(r["Grid_Size"]) for r in rows)
        for r in rows:
            if int(r["Grid_Size"]) == g:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                vals["_grid"] = [g]
                vals["_vgpr"] = [float(r["VGPR_Count"])]
                vals["_lds"] = [float(r["LDS_Block_Size"])]
                vals["_sgpr"] = [float(r["SGPR_Count"])]
    for k in sorted(vals):
        v = vals[k]
        print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(*sys.argv[1:])
