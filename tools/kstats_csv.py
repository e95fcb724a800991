#!/usr/bin/env python3
"""Per-kernel calls / average ms / share from a rocprofv3 --stats *kernel_stats.csv tree."""
import csv
import sys
from pathlib import Path

f = next(Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in list(csv.DictReader(open(f)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 6]:
    print(f"  {r['Name'][:40]:40s} calls {r['Calls']:>5s}  avg {float(r['AverageNs']) / 1e6:8.3f} ms  "
          f"total {float(r['TotalDurationNs']) / 1e6:9.1f} ms  {float(r['Percentage']):5.1f} %")
