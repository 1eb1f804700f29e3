#!/usr/bin/env python
"""Per-step kernel census of a rocprofv3 ``--kernel-trace`` database.

    python tools/prof_window.py run_results.db --anchor lstm_small_fwd [--skip 20] [--out x.md]

The anchor kernel (a substring of the kernel name) opens every training step;
the window runs from the ``--skip``-th anchor dispatch to the last one, so
start-up work (data upload, model init, kernel warm-up) is excluded.  Prints
dispatches and time per step for every kernel in the window.
"""
from __future__ import annotations

import argparse
import sqlite3
import sys

from prof_summary import short


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", required=True)
    ap.add_argument("--skip", type=int, default=20)
    ap.add_argument("--last", type=int, default=0, help="window = the last N anchor intervals (overrides --skip)")
    ap.add_argument("--first", type=int, default=0, help="window = N anchor intervals from the --skip-th anchor")
    ap.add_argument("--end-skip", type=int, default=0,
                    help="with --first: the window ENDS this many anchors before the last one")
    ap.add_argument("--sequence", type=int, default=0,
                    help="also list the dispatches of the first N anchor intervals of the window, in order")
    ap.add_argument("--timeline", type=int, default=0,
                    help="also list the first N anchor intervals as a timeline: start / end offsets and queue")
    ap.add_argument("--out")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    t0c = "start" if "start" in cols else ("begin" if "begin" in cols else None)
    if t0c is None:
        print("columns:", cols)
        return 1
    rows = c.execute(f"select name, {t0c}, duration from kernels order by {t0c}").fetchall()
    anchors = [r[1] for r in rows if a.anchor in r[0]]
    if len(anchors) <= a.skip + 1:
        print(f"only {len(anchors)} anchor dispatches")
        return 1
    skip = len(anchors) - 1 - a.last if a.last else a.skip
    end = min(skip + a.first, len(anchors) - 1) if a.first and not a.last else len(anchors) - 1
    if a.first and a.end_skip:
        end = len(anchors) - 1 - a.end_skip
        skip = max(end - a.first, 0)
    lo, hi = anchors[skip], anchors[end]
    steps = end - skip
    win = [r for r in rows if lo <= r[1] < hi]
    agg = {}
    for name, _, dur in win:
        n, t = agg.get(name, (0, 0))
        agg[name] = (n + 1, t + dur)
    span_us = (hi - lo) / 1e3
    out = [f"window: {steps} steps, {span_us:.1f} us wall ({span_us / steps:.2f} us/step)", "",
           "| kernel | dispatches/step | us/step |", "|---|---|---|"]
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append(f"| `{short(name)}` | {n / steps:.2f} | {t / 1e3 / steps:.2f} |")
    tot = sum(t for _, t in agg.values())
    out.append(f"\nGPU kernel time {tot / 1e3 / steps:.2f} us/step, {sum(n for n, _ in agg.values()) / steps:.2f} dispatches/step")
    if a.sequence:
        first = [r for r in win if anchors[skip] <= r[1] < anchors[min(skip + a.sequence, len(anchors) - 1)]]
        out += ["", "first window step, in dispatch order:", "", "| # | kernel | us |", "|---|---|---|"]
        out += [f"| {i} | `{short(n)}` | {d / 1e3:.2f} |" for i, (n, _, d) in enumerate(first)]
    if a.timeline:
        qc = next((q for q in ("queue_id", "stream_id") if q in cols), None)
        trows = c.execute(f"select name, {t0c}, duration{', ' + qc if qc else ''} from kernels order by {t0c}").fetchall()
        t_lo = anchors[skip]
        t_hi = anchors[min(skip + a.timeline, len(anchors) - 1)]
        out += ["", f"timeline of {a.timeline} window step(s) (us from the first anchor; queue = {qc}):", "",
                "| start | end | us | queue | kernel |", "|---|---|---|---|---|"]
        for r in trows:
            if t_lo <= r[1] < t_hi:
                q = r[3] if qc else "-"
                out.append(f"| {(r[1] - t_lo) / 1e3:.1f} | {(r[1] + r[2] - t_lo) / 1e3:.1f} | {r[2] / 1e3:.1f} | {q} | "
                           f"`{short(r[0])}` |")
    text = "\n".join(out)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    sys.exit(main())
