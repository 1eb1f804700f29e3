#!/usr/bin/env python
"""Overlap of collective kernels with persistent-recurrence kernels in a
rocprofv3 ``--kernel-trace`` database.

    python tools/prof_overlap.py run_results.db [--a persist] [--b Reduce]

For every dispatch whose name contains ``--b`` (default: the RCCL all-reduce
kernels) it reports the time it ran concurrently with dispatches whose name
contains ``--a`` (default: the grid-synced persistent recurrences), then a
timeline of the dispatches of both kinds.
"""
from __future__ import annotations

import argparse
import sqlite3
import sys

from prof_summary import short


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--a", default="persist")
    ap.add_argument("--b", default="Reduce")
    ap.add_argument("--rows", type=int, default=60)
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    t0c = "start" if "start" in cols else "begin"
    qc = next((q for q in ("queue_id", "stream_id") if q in cols), None)
    rows = c.execute(f"select name, {t0c}, duration{', ' + qc if qc else ''} from kernels order by {t0c}").fetchall()
    A = [(r[1], r[1] + r[2], r) for r in rows if a.a in r[0]]
    Bk = [(r[1], r[1] + r[2], r) for r in rows if a.b in r[0]]
    tot = sum(e - s for s, e, _ in Bk)
    ov = 0
    n_ov = 0
    for s, e, _ in Bk:
        o = sum(max(0, min(e, ae) - max(s, as_)) for as_, ae, _ in A)
        ov += o
        n_ov += o > 0
    out = [f"`{a.b}` dispatches: {len(Bk)}, {tot / 1e3:.1f} us; concurrent with a `{a.a}` dispatch: "
           f"{n_ov} of them, {ov / 1e3:.1f} us ({100.0 * ov / tot if tot else 0:.0f} %)",
           f"`{a.a}` dispatches: {len(A)}, {sum(e - s for s, e, _ in A) / 1e3:.1f} us", ""]
    ev = sorted(A + Bk, key=lambda x: x[0])
    if ev:
        t_lo = ev[0][0]
        out += ["| start us | end us | queue | kernel |", "|---|---|---|---|"]
        for s, e, r in ev[:a.rows]:
            out.append(f"| {(s - t_lo) / 1e3:.1f} | {(e - t_lo) / 1e3:.1f} | {r[3] if qc else '-'} | `{short(r[0])}` |")
    print("\n".join(out))


if __name__ == "__main__":
    sys.exit(main())
