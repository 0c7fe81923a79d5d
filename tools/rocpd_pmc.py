#!/usr/bin/env python3
"""Per-kernel PMC counter totals from a rocprofv3 SQLite database
(run_results.db): sum of each counter over the dispatches of every kernel,
plus mean dispatch time.

    python tools/rocpd_pmc.py gpurun_out/pmc1/run_results.db [kernel-substring]
"""
import collections
import sqlite3
import sys


def tables(cur):
    out = {}
    for (name,) in cur.execute("select name from sqlite_master where type='table'"):
        base = name.rsplit("_", 5)[0] if name.count("_") > 5 else name
        out[base] = name
    return out


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    con = sqlite3.connect(db)
    cur = con.cursor()
    t = tables(cur)
    names = {i: n for i, n in cur.execute(f"select id, name from {t['rocpd_info_pmc']}")}
    syms = {i: n for i, n in cur.execute(f"select id, display_name from {t['rocpd_info_kernel_symbol']}")}
    disp = {}
    for eid, kid, st, en in cur.execute(
            f"select event_id, kernel_id, start, end from {t['rocpd_kernel_dispatch']}"):
        disp[eid] = (syms.get(kid, str(kid)), en - st)
    agg = collections.defaultdict(collections.Counter)
    seen = collections.defaultdict(set)
    for eid, pid, val in cur.execute(f"select event_id, pmc_id, value from {t['rocpd_pmc_event']}"):
        if eid not in disp:
            continue
        k, ns = disp[eid]
        if filt and filt not in k:
            continue
        agg[k][names.get(pid, str(pid))] += val
        if eid not in seen[k]:
            seen[k].add(eid)
            agg[k]["_ns"] += ns
    for k, c in agg.items():
        n = len(seen[k])
        print(f"{k[:90]}  dispatches={n} mean_us={c['_ns'] / n / 1e3:.1f}")
        for name in sorted(x for x in c if x != "_ns"):
            print(f"    {name:28s} {c[name] / n:16.1f}")


if __name__ == "__main__":
    main()
