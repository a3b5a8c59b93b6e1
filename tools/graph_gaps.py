#!/usr/bin/env python
"""Busy vs idle time of the GPU across the last ``--kernels`` dispatches of a
rocprofv3 kernel trace (rocpd sqlite): sum of kernel durations, wall span from
first start to last end, and the largest inter-kernel gaps.  Used on the
hipGraph-replayed UNet step to price launch bubbles:

    rocprofv3 --kernel-trace -d /tmp/kt -o k -- python tools/abstep.py --rounds 1 --iters 3
    python tools/graph_gaps.py /tmp/kt/k_results.db --marker timestep_emb
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernels", type=int, default=354)
    ap.add_argument("--marker", default="", help="kernel name starting each step: analyse the last full step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    if a.marker:
        idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
        if len(idx) >= 2:
            rows = rows[idx[-2]:idx[-1]]
            print(f"last full step between markers: {len(rows)} kernels")
    else:
        rows = rows[-a.kernels:]
    busy = sum(e - s for _, s, e in rows)
    span = rows[-1][2] - rows[0][1]
    gaps = []
    for (n0, _s0, e0), (n1, s1, _e1) in zip(rows, rows[1:]):
        gaps.append((s1 - e0, n0[:50], n1[:50]))
    gaps.sort(reverse=True)
    print(f"{len(rows)} kernels: busy {busy / 1e6:.3f} ms, span {span / 1e6:.3f} ms, "
          f"idle {(span - busy) / 1e6:.3f} ms ({100 * (span - busy) / span:.1f} %), "
          f"mean gap {sum(g for g, *_ in gaps) / max(1, len(gaps)) / 1e3:.2f} us")
    for g, n0, n1 in gaps[:15]:
        print(f"  {g / 1e3:8.2f} us  {n0}  ->  {n1}")


if __name__ == "__main__":
    main()
