"""Per-kernel effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) from a rocprofv3
--pmc GRBM_GUI_ACTIVE ... --kernel-trace run.  usage: python tools/clock_summary.py DIR"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(kt))}
vals = collections.defaultdict(dict)
for r in csv.DictReader(open(cc)):
    vals[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    vals[r["Dispatch_Id"]]["name"] = r["Kernel_Name"]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for did, v in vals.items():
    t = tr.get(did)
    if t is None or "GRBM_GUI_ACTIVE" not in v:
        continue
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9
    a = agg[v["name"][:90]]
    a[0] += 1
    a[1] += dur
    a[2] += v["GRBM_GUI_ACTIVE"] / 8
tot = sum(a[1] for a in agg.values())
for name, (n, dur, cyc) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"{n:5d} {dur * 1e3:9.3f} ms {dur / tot * 100:5.1f}%  clk {cyc / dur / 1e9:5.3f} GHz  {name}")
