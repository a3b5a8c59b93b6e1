#!/usr/bin/env python
"""Per-kernel mean PMC counter values from rocprofv3 rocpd databases.

    python tools/pmc_summary.py gpurun_out/pmcg_x_1/p_results.db [more.db ...] [--filter gemm]
"""
import sqlite3
import sys
from collections import defaultdict


def main(paths, filt=""):
    agg = defaultdict(lambda: defaultdict(list))
    for p in paths:
        c = sqlite3.connect(p)
        rows = c.execute("select name, dispatch_id, counter_name, sum(counter_value), duration from pmc_events "
                         "group by dispatch_id, counter_name").fetchall()
        for name, _d, cn, v, dur in rows:
            if filt in name:
                agg[name][cn].append(v)
                agg[name]["_dur_ns"].append(dur)
    for name, cs in agg.items():
        print(name[:120])
        for cn in sorted(cs):
            v = cs[cn]
            print(f"   {cn:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--filter")]
    filt = ""
    for a in sys.argv[1:]:
        if a.startswith("--filter="):
            filt = a.split("=", 1)[1]
    main(args, filt)
