#!/usr/bin/env python
"""Per-denoising-step GPU busy vs wall time inside a whole job trace
(rocprofv3 --kernel-trace rocpd sqlite): steps are delimited by a marker
kernel that runs once at the head of every UNet evaluation (the timestep
embedding).  Reports median busy / wall / idle per step and where the idle
time sits (which kernel pairs border the largest gaps, summed over steps).

    python tools/jobgaps.py gpurun_out/prof_x/.../prof_results.db --marker timestep_emb
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import collections
import glob
import sqlite3
import statistics


def load(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    return c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="timestep_emb")
    ap.add_argument("--steps", type=int, default=50, help="steps per job (last job analysed)")
    a = ap.parse_args()
    dbs = glob.glob(a.db) or [a.db]
    rows = load(dbs[0])
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    # the last job's steps: the last `steps` markers (+ the kernels up to the next marker / end)
    idx = idx[-a.steps:]
    busy, wall = [], []
    pair_idle = collections.Counter()
    for k, i0 in enumerate(idx):
        i1 = idx[k + 1] if k + 1 < len(idx) else None
        seg = rows[i0:i1] if i1 is not None else rows[i0:i0 + (idx[1] - idx[0] if len(idx) > 1 else 1)]
        b = sum(e - s for _, s, e in seg)
        w = (rows[i1][1] if i1 is not None else seg[-1][2]) - seg[0][1]
        busy.append(b)
        wall.append(w)
        full = rows[i0:(i1 + 1) if i1 is not None else i0 + len(seg)]
        for (n0, _s0, e0), (n1, s1, _e1) in zip(full, full[1:]):
            pair_idle[(n0[:48], n1[:48])] += max(0, s1 - e0)
    n = len(idx)
    print(f"{n} steps: busy median {statistics.median(busy) / 1e6:.3f} ms, wall median "
          f"{statistics.median(wall) / 1e6:.3f} ms, idle median "
          f"{statistics.median([w - b for w, b in zip(wall, busy)]) / 1e3:.1f} us per step")
    if n:
        print(f"kernels per step: {idx[1] - idx[0] if n > 1 else 'n/a'}")
    print("largest idle contributors (summed over steps, us):")
    for (n0, n1), g in pair_idle.most_common(15):
        print(f"  {g / 1e3:9.1f}  {n0}  ->  {n1}")


if __name__ == "__main__":
    main()
