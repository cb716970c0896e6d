"""Aggregate rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KiB and count L2 <-> fabric (Infinity Cache + HBM)
traffic.  On gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads
(MI355X_MICROARCH.md, HBM section), so it is doubled here.  Prints JSON:
{kernel symbol: {"launches", "fetch_bytes", "write_bytes", "bytes_per_launch"}}.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(pattern, counter):
    acc = collections.defaultdict(lambda: [0, 0.0])
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            a = acc[r["Kernel_Name"]]
            a[0] += 1
            a[1] += float(r["Counter_Value"]) * 1024.0
    return acc


def main():
    d = sys.argv[1]
    fe = load(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    fe.update(load(os.path.join(d, "fetch", "*counter_collection.csv"), "FETCH_SIZE"))
    wr = load(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    wr.update(load(os.path.join(d, "write", "*counter_collection.csv"), "WRITE_SIZE"))
    out = {}
    for k in fe:
        n_f, b_f = fe[k]
        n_w, b_w = wr.get(k, [0, 0.0])
        fetch = 2.0 * b_f / max(n_f, 1)
        write = b_w / max(n_w, 1)
        out[k] = {"launches": n_f, "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
