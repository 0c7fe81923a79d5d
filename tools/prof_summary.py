#!/usr/bin/env python3
"""Per-kernel time summary of a rocprofv3 (rocpd sqlite) kernel trace:
    python tools/prof_summary.py gpurun_out/prof_bert/bert_results.db [--last N] [--top K]
``--last N`` keeps only the last N dispatches of the trace (e.g. the timed
steps after warm-up / autotuning).  Prints a table and writes nothing."""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=int, default=0,
                    help="keep the last N optimizer steps (segments ending at an adam / sgd update kernel)")
    ap.add_argument("--marker", default="",
                    help="regex of a kernel launched exactly once per step (e.g. the loss kernel) that marks the "
                         "step boundaries instead of the last update kernel (steps with several update launches)")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end from kernels order by start").fetchall()
    if a.last:
        rows = rows[-a.last:]
    if a.steps:
        # a step ends with the same optimizer-update kernel every time: the
        # last update kernel of the trace marks the step boundaries
        upd = [r[0] for r in rows if re.search(a.marker or r"adam|sgd", r[0])]
        marks = [i for i, r in enumerate(rows) if upd and r[0] == upd[-1]]
        n = min(a.steps, len(marks) - 1)
        if n > 0:
            rows = rows[marks[-n - 1] + 1:marks[-1] + 1]
        print(f"last {n} steps: {len(rows)} dispatches")
    span = (rows[-1][2] - rows[0][1]) / 1e6 if rows else 0.0
    tot = collections.Counter()
    cnt = collections.Counter()
    for name, s, e in rows:
        k = short(name)
        tot[k] += (e - s) / 1e6
        cnt[k] += 1
    busy = sum(tot.values())
    print(f"dispatches {len(rows)}  kernel time {busy:.2f} ms  wall span {span:.2f} ms")
    print(f"{'ms':>9} {'%':>6} {'n':>6}  kernel")
    for k, v in tot.most_common(a.top):
        print(f"{v:9.3f} {100 * v / busy:6.2f} {cnt[k]:6d}  {k}")


if __name__ == "__main__":
    main()
