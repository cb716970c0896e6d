"""Aggregate rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KiB and count L2 <-> fabric (Infinity Cache + HBM)
traffic.  On gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads
(MI355X_MICROARCH.md, HBM section), so it is doubled here -- the tally of 128-B line
requests.  tools/probe/fetch_calib.hip measured the other widths on a 2 GiB buffer (run
r4b): 128-B lines (a float4 stream, or a line's two 64-B halves read by two blocks of one XCD)
tally 1/2; isolated 64-B pieces tally 1:1; 16-B pieces are fetched as 64-B sectors (4x the
requested bytes, tallied 1:1).  Kernels whose reads are isolated 64-B pieces (PIECE64 below:
the narrow ConvT's 16-channel chunks of 128-channel rows) are therefore not doubled.  Prints JSON:
{kernel symbol: {"launches", "fetch_bytes", "write_bytes", "bytes_per_launch"}}.
"""
import collections
import csv
import glob
import json
import os
import sys


# kernels whose global reads are isolated 64-B pieces (FETCH_SIZE tallied 1:1)
PIECE64 = ("convt2_narrow_mfma",)


def load(pattern, counter, by_grid=False):
    acc = collections.defaultdict(lambda: [0, 0.0])
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            a = acc[(r["Kernel_Name"], int(r["Grid_Size"])) if by_grid else r["Kernel_Name"]]
            a[0] += 1
            a[1] += float(r["Counter_Value"]) * 1024.0
    return acc


def main():
    d = sys.argv[1]
    bg = "--by-grid" in sys.argv  # per (symbol, grid size): the launches of one layer shape
    fe = load(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE", bg)
    fe.update(load(os.path.join(d, "fetch", "*counter_collection.csv"), "FETCH_SIZE", bg))
    wr = load(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE", bg)
    wr.update(load(os.path.join(d, "write", "*counter_collection.csv"), "WRITE_SIZE", bg))
    out = {}
    for k in fe:
        n_f, b_f = fe[k]
        n_w, b_w = wr.get(k, [0, 0.0])
        fetch = (1.0 if any(p in k for p in PIECE64) else 2.0) * b_f / max(n_f, 1)
        write = b_w / max(n_w, 1)
        key = f"{k[0]} @grid {k[1]}" if bg else k
        if bg and "gemm" not in k[0]:
            continue
        out[key] = {"launches": n_f, "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
