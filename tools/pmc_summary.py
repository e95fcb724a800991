#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files under a directory."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    for k in ("k_trace<true>", "k_trace<false>", "k_shade", "k_raygen", "k_shadow_resolve", "k_resolve_pixels",
              "k_pixel_sets", "k_debug", "k_pick"):
        if k.replace("<true>", "ILb1E").replace("<false>", "ILb0E") in name or k in name:
            return k
    return name[:40]


def main(root):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in Path(root).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                c = row.get("Counter_Name", "")
                vals[k][c] += float(row.get("Counter_Value", 0) or 0)
                disp[k][c].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for k in sorted(vals):
        print(k)
        for c in sorted(vals[k]):
            n = max(1, len(disp[k][c]))
            print(f"  {c:32s} total {vals[k][c]:.6g}  per-dispatch {vals[k][c] / n:.6g}  ({n} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1])
