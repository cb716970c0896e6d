#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite .db or kernel_stats.csv).

usage: python profiles/summarize.py <run_results.db | dir> [top_n]
Prints: kernel symbol, calls, total ms, avg us, share of GPU kernel time.
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in c.execute(f"pragma table_info({ks})")]
    name_col = "display_name" if "display_name" in cols else ("kernel_name" if "kernel_name" in cols else "name")
    rows = c.execute(f"select s.{name_col}, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        a = agg.setdefault(name, [0, 0])
        a[0] += 1
        a[1] += dur
    return agg


def from_csv(path):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[r["Name"]] = [int(r["Calls"]), float(r["TotalDurationNs"])]
    return agg


def main():
    src = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
        agg = from_db(dbs[0]) if dbs else from_csv(csvs[0])
    else:
        agg = from_db(src) if src.endswith(".db") else from_csv(src)
    total = sum(v[1] for v in agg.values())
    print(f"{'calls':>7} {'total_ms':>10} {'avg_us':>10} {'share':>7}  kernel")
    for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:7d} {ns / 1e6:10.3f} {ns / n / 1e3:10.2f} {100 * ns / total:6.2f}%  {name[:140]}")
    print(f"total GPU kernel time: {total / 1e6:.3f} ms over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main()
