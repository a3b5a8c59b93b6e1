#!/usr/bin/env python
"""Per-kernel mean PMC counter values from rocprofv3 rocpd databases, plus a
derived table ranked by total time:

    python tools/pmc_summary.py gpurun_out/pmcg_x_1/p_results.db [more.db ...] [--filter=gemm] [--raw]

Derived columns (when the pass collected them):
    mfma_util    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * CUs)
    ldsconf/inst SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS
    valu/mfma    SQ_INSTS_VALU / SQ_INSTS_MFMA
    TB/s         (FETCH_SIZE + WRITE_SIZE) KiB / duration
"""
import sqlite3
import sys
from collections import defaultdict

CUS = 256


def collect(paths, filt=""):
    agg = defaultdict(lambda: defaultdict(list))
    for p in paths:
        c = sqlite3.connect(p)
        rows = c.execute("select name, dispatch_id, counter_name, sum(counter_value), duration from pmc_events "
                         "group by dispatch_id, counter_name").fetchall()
        seen = set()
        for name, d, cn, v, dur in rows:
            if filt in name:
                agg[name][cn].append(v)
                if (p, d) not in seen:
                    seen.add((p, d))
                    agg[name]["_dur_ns"].append(dur)
    return agg


def mean(v):
    return sum(v) / len(v) if v else 0.0


def derived(agg, top=40):
    out = []
    for name, cs in agg.items():
        m = {k: mean(v) for k, v in cs.items()}
        tot = sum(cs["_dur_ns"])
        row = {"name": name, "calls": len(cs["_dur_ns"]), "mean_us": m["_dur_ns"] / 1e3, "total_us": tot / 1e3}
        if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            row["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] * CUS)
        if m.get("SQ_INSTS_LDS"):
            row["ldsconf/inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
        if m.get("SQ_INSTS_MFMA"):
            row["valu/mfma"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_INSTS_MFMA"]
        if "FETCH_SIZE" in m and m["_dur_ns"]:
            row["TB/s"] = (m["FETCH_SIZE"] + m.get("WRITE_SIZE", 0.0)) * 1024 / m["_dur_ns"] / 1e3
        out.append(row)
    out.sort(key=lambda r: -r["total_us"])
    cols = [c for c in ("mfma_util", "ldsconf/inst", "valu/mfma", "TB/s") if any(c in r for r in out)]
    print(f"{'total_us':>10s} {'calls':>6s} {'mean_us':>8s} " + " ".join(f"{c:>12s}" for c in cols) + "  kernel")
    for r in out[:top]:
        vals = " ".join(f"{r[c]:12.3f}" if c in r else f"{'-':>12s}" for c in cols)
        print(f"{r['total_us']:10.1f} {r['calls']:6d} {r['mean_us']:8.1f} {vals}  {r['name'][:100]}")


def main(argv):
    paths = [a for a in argv if not a.startswith("--")]
    filt = next((a.split("=", 1)[1] for a in argv if a.startswith("--filter=")), "")
    agg = collect(paths, filt)
    derived(agg)
    if "--raw" in argv:
        print("\n# raw per-kernel means")
        for name, cs in agg.items():
            print(name[:120])
            for cn in sorted(cs):
                print(f"   {cn:28s} {mean(cs[cn]):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
