#!/usr/bin/env python3
"""Per-dispatch durations of a rocprofv3 kernel trace grouped by (kernel, grid, block): count,
mean and min microseconds -- which call shapes of one symbol are slow.
usage: python tools/trace_by_grid.py run_kernel_trace.csv [substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if pats and not any(p in name for p in pats):
                continue
            key = (name.split("(")[0][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):5d} {sum(v) / len(v):8.2f} {min(v):8.2f}  {k[0]} grid=({k[1]},{k[2]},{k[3]}) wg={k[4]}")


if __name__ == "__main__":
    main()
