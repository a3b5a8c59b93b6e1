#!/usr/bin/env python
"""Per-kernel time difference between two rocpd databases (e.g. two A/B arms of
tools/abstep.py traced by tools/gpu/prof_ab.sh), normalised per --div runs.

    python tools/rocpd_diff.py A/prof_results.db B/prof_results.db --div 10
"""
import argparse
import sqlite3
from collections import defaultdict


def load(path):
    c = sqlite3.connect(path)
    d = defaultdict(lambda: [0, 0.0])
    for n, s, e in c.execute("select name, start, end from kernels"):
        k = n.split("(")[0][:90]
        d[k][0] += 1
        d[k][1] += (e - s) / 1e3
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--div", type=float, default=1.0)
    a = ap.parse_args()
    A, B = load(a.a), load(a.b)
    rows = []
    for k in set(A) | set(B):
        ta, tb = A[k][1] / a.div, B[k][1] / a.div
        rows.append((tb - ta, k, A[k][0], B[k][0], ta, tb))
    print(f"total A {sum(r[4] for r in rows):.1f} us  B {sum(r[5] for r in rows):.1f} us (per unit)")
    for d, k, ca, cb, ta, tb in sorted(rows, key=lambda r: -abs(r[0]))[:25]:
        print(f"{d:+9.1f} us  A {ta:9.1f} ({ca:5d})  B {tb:9.1f} ({cb:5d})  {k}")


if __name__ == "__main__":
    main()
