#!/usr/bin/env python3
"""Per-item dynamic instruction counts from a rocprofv3 --pmc counter_collection.csv tree and the
bench JSON of the same run (items: shade = closest queries, trace<false> = closest, trace<true>
= shadow). Counts are wave instructions per 64 items."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

f = next(Path(sys.argv[1]).rglob("*counter_collection.csv"))
b = json.loads(Path(sys.argv[2]).read_text().strip().splitlines()[-1])
sums = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    name = "k_shade" if "k_shade" in k else "k_trace<false>" if "k_trace<false>" in k else \
        "k_trace<true>" if "k_trace<true>" in k else None
    if name:
        sums[name][r["Counter_Name"]] += float(r["Counter_Value"])
items = {"k_shade": b["rays_closest"], "k_trace<false>": b["rays_closest"], "k_trace<true>": b["rays_shadow"]}
for k, c in sums.items():
    n = items[k] / 64.0
    print(f"  {k:15s} items {items[k]:.3g}  per 64 items: VALU {c['SQ_INSTS_VALU'] / n:8.1f}  "
          f"SALU {c['SQ_INSTS_SALU'] / n:8.1f}  VMEM_RD {c['SQ_INSTS_VMEM_RD'] / n:6.1f}")
