"""Summarise a rocprofv3 --kernel-trace database (rocpd SQLite) into the --stats CSV layout
("Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev").

usage: python tools/rocprof_summary.py <run_results.db> [out.csv]
"""
import csv
import sqlite3
import sys

import numpy as np


def summarize(db):
    c = sqlite3.connect(db)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        rows.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in rows.values())
    out = []
    for name, d in rows.items():
        d = np.asarray(d, dtype=np.float64)
        out.append([name, len(d), int(d.sum()), d.mean(), 100.0 * d.sum() / total, int(d.min()), int(d.max()), d.std()])
    out.sort(key=lambda r: -r[2])
    return out


def main():
    rows = summarize(sys.argv[1])
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 3), round(r[4], 2), r[5], r[6], round(r[7], 3)])


if __name__ == "__main__":
    main()
