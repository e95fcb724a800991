#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace --stats output (rocpd SQLite .db, or the CSV
kernel_stats file) into a per-kernel table (calls, total/avg/min/max us, % of GPU time)."""
import csv
import sqlite3
import sys
from pathlib import Path


def from_db(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    ext = {}
    try:
        for name, mn, mx in c.execute("select name, min(duration), max(duration) from kernels group by name"):
            ext[name] = (mn, mx)
    except sqlite3.Error:
        pass
    return [(n, calls, tot, avg, ext.get(n, (None, None))[0], ext.get(n, (None, None))[1], pct)
            for n, calls, tot, avg, pct in rows]


def main(src, out):
    src = Path(src)
    dbs = [src] if src.suffix == ".db" else sorted(src.rglob("*.db"))
    rows = from_db(dbs[0])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        # top_kernels reports microseconds; the per-dispatch kernels view nanoseconds
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "percent"])
        for n, calls, tot, avg, mn, mx, pct in rows:
            f_ = lambda v: "" if v is None else f"{v / 1000.0:.3f}"  # noqa: E731
            w.writerow([n, calls, f"{tot:.1f}", f"{avg:.3f}", f_(mn), f_(mx), f"{pct:.2f}"])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
