#!/usr/bin/env python3
"""Kernel timeline of the last render in a rocprofv3 kernel trace (tools/batches/r04/gpu_round4_c4b.sh):
the job's span, how much of it the GPU runs kernels on one lane, on both, or on none, the
small (near-empty) launches and the tail after the last raygen.

usage: python tools/c4_timeline.py <rocprofv3 output dir> [--job k]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
f = next(d.rglob("*kernel_trace.csv"))
rows = list(csv.DictReader(open(f)))
lane_key = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[lane_key],
              int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)) for r in rows), key=lambda k: k[0])
# a job starts with its parameter / camera uploads (copyBuffer kernels); without them, by an
# idle gap > 2 ms. --job k picks the k-th job from the end (default the last).
k = int(sys.argv[sys.argv.index("--job") + 1]) if "--job" in sys.argv else 1
cuts = [i for i, x in enumerate(ks) if "copyBuffer" in x[2] and (i == 0 or "copyBuffer" not in ks[i - 1][2])]
if len(cuts) < k:
    cuts, end = [0], 0
    for i, x in enumerate(ks):
        if i and x[0] - end > 2_000_000:
            cuts.append(i)
        end = max(end, x[1])
first = cuts[-k]
stop = cuts[-k + 1] if k > 1 else len(ks)
job = ks[first:stop]
print(f"{len(cuts)} jobs in the trace; job {len(cuts) - k + 1}")
t0 = job[0][0]
t1 = max(k[1] for k in job)
span = t1 - t0
# coverage: sweep over start/end events, time with 0 / 1 / >=2 kernels in flight
ev = sorted([(k[0], 1) for k in job] + [(k[1], -1) for k in job])
cover = defaultdict(int)
cur, last = 0, t0
for t, dlt in ev:
    cover[min(cur, 2)] += t - last
    cur += dlt
    last = t
short = lambda n: n.split("(")[0].replace("void ", "").replace("yrt::", "")
by = defaultdict(lambda: [0, 0, 0, 0])  # calls, ns, calls < 20 us, ns in those
for s, e, n, _, _ in job:
    b = by[short(n)]
    b[0] += 1
    b[1] += e - s
    if e - s < 20000:
        b[2] += 1
        b[3] += e - s
last_raygen = max((k[1] for k in job if "k_raygen" in k[2]), default=t0)
lanes = sorted({k[3] for k in job})
print(f"trace {f.name}: {len(job)} kernels in the last job, span {span / 1e6:.2f} ms, lanes {lanes}")
print(f"  busy on 0 lanes {cover[0] / 1e6:.2f} ms, on 1 lane {cover[1] / 1e6:.2f} ms, on >=2 {cover[2] / 1e6:.2f} ms")
print(f"  first kernel -> last raygen end {(last_raygen - t0) / 1e6:.2f} ms; tail after it {(t1 - last_raygen) / 1e6:.2f} ms")
for n, (c, ns, sc, sns) in sorted(by.items(), key=lambda x: -x[1][1]):
    print(f"  {n:32s} {c:5d} calls {ns / 1e6:8.2f} ms   <20us: {sc:4d} calls {sns / 1e6:6.3f} ms")
# per-lane: idle gaps between consecutive kernels of a lane
for ln in lanes:
    lk = [k for k in job if k[3] == ln]
    gaps = [b[0] - a[1] for a, b in zip(lk, lk[1:])]
    busy = sum(k[1] - k[0] for k in lk)
    print(f"  lane {ln}: {len(lk)} kernels, busy {busy / 1e6:.2f} ms, gaps {sum(gaps) / 1e6:.2f} ms "
          f"(median {sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.1f} us), first {(lk[0][0] - t0) / 1e6:.2f} ms, "
          f"last end {(lk[-1][1] - t0) / 1e6:.2f} ms")
