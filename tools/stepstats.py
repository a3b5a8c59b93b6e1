#!/usr/bin/env python
"""Kernel time breakdown of ONE hipGraph-replayed UNet step from a rocpd database
(the window between the last two timestep-embedding launches).

    python tools/stepstats.py gpurun_out/profab_x/prof_results.db [substring]
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import collections
import sqlite3
import sys


def main(path, filt=""):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    ts = [r[1] for r in rows if r[0].startswith("timestep_emb")]
    win = [r for r in rows if ts[-2] <= r[1] < ts[-1]]
    d = collections.defaultdict(lambda: [0, 0])
    for n, s, e in win:
        d[n][0] += 1
        d[n][1] += e - s
    print(f"kernels {len(win)}  busy {sum(v[1] for v in d.values()) / 1e3:.1f} us  "
          f"wall {(win[-1][2] - win[0][1]) / 1e3:.1f} us")
    for n, v in sorted(d.items(), key=lambda kv: -kv[1][1]):
        if filt in n:
            print(f"{v[1] / 1e3:8.1f} us {v[0]:4d}  {n[:100]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
