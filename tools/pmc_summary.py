#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel category:
MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x SIMDs, the
MfmaUtil derived metric), achieved bf16 MFMA TFLOP/s from
SQ_INSTS_VALU_MFMA_MOPS_BF16 (x512 FLOP) over the dispatch time, and LDS
bank-conflict rate (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE); with a
FETCH_SIZE pass, the achieved HBM read bandwidth.

    python tools/pmc_summary.py gpurun_out/pmc/bert1/run_counter_collection.csv [--simds 1024] [--xcds 8] [--raw]
"""
import collections
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def category(name: str) -> str:
    """Kernel name without arguments; hipBLASLt kernels grouped by macro tile."""
    if "Cijk_" in name:
        m = re.search(r"MT\d+x\d+x\d+", name)
        return f"hipBLASLt gemm ({m.group(0) if m else '?'})"
    return short(name)


def main():
    path = sys.argv[1]
    simds = int(sys.argv[sys.argv.index("--simds") + 1]) if "--simds" in sys.argv else 1024
    xcds = int(sys.argv[sys.argv.index("--xcds") + 1]) if "--xcds" in sys.argv else 8
    disp = collections.defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            d = disp[(r["Dispatch_Id"], r["Kernel_Name"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.Counter())
    for (_, name), d in disp.items():
        a = agg[category(name)]
        a["n"] += 1
        a["ns"] += d["_ns"]
        for k, v in d.items():
            if not k.startswith("_"):
                a[k] += v
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])
    has_fetch = any("FETCH_SIZE" in a for a in agg.values())
    print(f"{'kernel (category)':60s} {'calls':>6s} {'ms':>8s} {'MFMA busy%':>10s} {'bf16 TF/s':>9s} {'LDS confl%':>10s}"
          + (f" {'HBM rd GB/s':>11s}" if has_fetch else ""))
    for name, a in rows[:30]:
        gui = a.get("GRBM_GUI_ACTIVE", 0) / xcds
        busy = 100.0 * a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * simds) if gui else 0.0
        tf = a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512 / (a["ns"] * 1e-9) / 1e12 if a["ns"] else 0.0
        lds = a.get("SQ_LDS_IDX_ACTIVE", 0)
        confl = 100.0 * a.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0.0
        line = f"{name[:60]:60s} {a['n']:6d} {a['ns'] / 1e6:8.2f} {busy:10.1f} {tf:9.1f} {confl:10.1f}"
        if has_fetch:  # FETCH_SIZE is in KiB
            line += f" {a.get('FETCH_SIZE', 0) * 1024 / (a['ns'] * 1e-9) / 1e9 if a['ns'] else 0.0:11.1f}"
        print(line)
    if "--raw" in sys.argv:   # every counter, mean per dispatch
        for name, a in rows[:30]:
            print(f"{name[:90]}  dispatches={a['n']} mean_us={a['ns'] / a['n'] / 1e3:.1f}")
            for k in sorted(x for x in a if x not in ("n", "ns")):
                print(f"    {k:32s} {a[k] / a['n']:18.1f}")


if __name__ == "__main__":
    main()
