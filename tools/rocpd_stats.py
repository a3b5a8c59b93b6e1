#!/usr/bin/env python
"""Per-kernel stats CSV (rocprofv3 --stats layout) from a rocpd sqlite database.

    python tools/rocpd_stats.py gpurun_out/prof_x/prof_results.db > profiles/x_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main(path, out=sys.stdout):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    d = defaultdict(list)
    for n, s, e in rows:
        d[n].append(e - s)
    tot = sum(sum(v) for v in d.values())
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([n, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 3), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
