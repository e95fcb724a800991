#!/usr/bin/env python3
"""Effective GPU clock per kernel from one rocprofv3 pass with `--pmc GRBM_GUI_ACTIVE
--kernel-trace`: GRBM_GUI_ACTIVE (busy cycles, summed over the 8 XCDs) / 8 / the dispatch's
duration. Two builds whose kernel runs the same instructions on the same work but takes longer
per launch either wait more on memory (same cycles per unit of work, fewer done) or ran at a
lower clock (same cycles, longer time); this tells the two apart.

    python tools/clock_check.py <rocprofv3 output dir> [top N kernels]
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 6
times = {}
for f in d.rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        times[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
cyc = {}
name = {}
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        k = r["Dispatch_Id"]
        cyc[k] = cyc.get(k, 0.0) + float(r["Counter_Value"] or 0)
        name[k] = r["Kernel_Name"]
        if k not in times and r.get("Start_Timestamp") and r.get("End_Timestamp"):
            times[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = defaultdict(lambda: [0, 0.0, 0.0])
for k, c in cyc.items():
    if k not in times or times[k] <= 0:
        continue
    a = agg[name[k][:60]]
    a[0] += 1
    a[1] += c / 8.0
    a[2] += times[k]
rows = sorted(agg.items(), key=lambda kv: -kv[1][2])[:top]
for n, (cnt, c, t) in rows:
    print(f"{n:60s} dispatches {cnt:5d}  ms/launch {t / cnt * 1e3:8.3f}  Mcycles/launch {c / cnt * 1e-6:8.3f}  "
          f"clock {c / t * 1e-6:7.1f} MHz")
