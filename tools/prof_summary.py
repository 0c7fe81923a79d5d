#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv into categories (short names).

    python tools/prof_summary.py gpurun_out/prof/bert_kernel_stats.csv [--steps N]
    python tools/prof_summary.py gpurun_out/prof/bert_results.db --steps 10 --window-ms 540

``--window-ms W`` (rocpd .db only) keeps the dispatches that START within
the last W ms of the trace: the timed steps of a bench run, excluding
autotuning / warm-up kernels.
"""
import csv
import json
import re
import sys


def category(name: str) -> str:
    n = name
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        out = "S" if "_BSS_" in n or "_SS_" in n else "B"
        mt = re.search(r"MT(\d+x\d+x\d+)", n)
        return f"hipBLASLt gemm ({'fp32' if out == 'S' else 'bf16'} out, MT{mt.group(1) if mt else '?'})"
    m = re.search(r"ffk::(?:\(anonymous namespace\)::)?([A-Za-z0-9_]+)", n)
    if m:
        return "ffk::" + m.group(1)
    m = re.search(r"_ZN3ffk\d+([A-Za-z0-9_]+?)(?:I|E)", n)
    if m:
        return "ffk::" + m.group(1)
    m = re.search(r"at::native::[^<(]*?(\w+Functor\w*|\w+_kernel\w*)", n)
    if m:
        return "torch::" + m.group(1)
    if "rccl" in n.lower() or "nccl" in n.lower():
        return "rccl::" + n.split("(")[0][:60]
    return n.split("(")[0][:80]


def main():
    path = sys.argv[1]
    steps = 1
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    agg = {}
    total = 0

    def add(name, calls, ns):
        nonlocal total
        d = agg.setdefault(category(name), {"calls": 0, "ns": 0})
        d["calls"] += int(calls)
        d["ns"] += int(ns)
        total += int(ns)

    if path.endswith(".db"):
        # rocprofv3 rocpd (SQLite) output: per-dispatch durations in ns
        import sqlite3

        con = sqlite3.connect(path)
        where = ""
        if "--window-ms" in sys.argv:
            w = float(sys.argv[sys.argv.index("--window-ms") + 1])
            (end,) = con.execute("select max(end) from kernels").fetchone()
            where = f" where start >= {int(end - w * 1e6)}"
        for name, calls, ns in con.execute(f"select name, count(*), sum(duration) from kernels{where} group by name"):
            add(name, calls, ns)
    else:
        with open(path) as f:
            for row in csv.DictReader(f):
                add(row["Name"], row["Calls"], row["TotalDurationNs"])
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])
    print(f"{'kernel (category)':70s} {'calls/step':>10s} {'ms/step':>9s} {'%':>6s}")
    for k, v in rows:
        print(f"{k[:70]:70s} {v['calls'] / steps:10.1f} {v['ns'] / 1e6 / steps:9.3f} {100.0 * v['ns'] / total:6.2f}")
    print(f"{'TOTAL':70s} {'':10s} {total / 1e6 / steps:9.3f}")
    if "--json" in sys.argv:
        print(json.dumps({k: {"calls_per_step": v["calls"] / steps, "ms_per_step": v["ns"] / 1e6 / steps}
                          for k, v in rows}))


if __name__ == "__main__":
    main()
