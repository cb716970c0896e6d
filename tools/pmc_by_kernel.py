#!/usr/bin/env python3
"""Mean PMC counter values per dispatch of the kernels matching a substring, grouped by grid
size, from a rocprofv3 --pmc csv directory.  usage: pmc_by_kernel.py DIR SUBSTRING"""
import collections
import csv
import glob
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, grid), cs in sorted(acc.items()):
        vals = "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
        print(f"{k} grid={grid}: {vals}")


if __name__ == "__main__":
    main()
