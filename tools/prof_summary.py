#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace`` rocpd database as a markdown table.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--out profiles/x.md]

Per kernel: calls, total / mean / min duration (us), share of GPU time, grid,
workgroup, VGPR / AGPR / SGPR counts and LDS bytes (from the dispatch records).
"""
from __future__ import annotations

import argparse
import re
import sqlite3
import sys


def short(name: str, width: int = 90) -> str:
    name = re.sub(r"pdrnn::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(Pdrnn\w+\)", "", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def summarise(db: str, top: int = 25) -> str:
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(grid_x), max(workgroup_x),"
        " max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size) from kernels"
        " group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = ["| kernel | calls | total us | mean us | min us | % | grid | wg | vgpr | agpr | sgpr | lds B |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:top]:
        name, n, tot, avg, mn, gx, wx, vg, ag, sg, lds = r
        out.append(f"| `{short(name)}` | {n} | {tot / 1e3:.1f} | {avg / 1e3:.2f} | {mn / 1e3:.2f} | "
                   f"{100 * tot / total:.1f} | {gx} | {wx} | {vg} | {ag} | {sg} | {lds} |")
    out.append(f"\nTotal GPU kernel time: {total / 1e3:.1f} us over {sum(r[1] for r in rows)} dispatches")
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    a = ap.parse_args(argv)
    text = summarise(a.db, a.top)
    if a.title:
        text = f"# {a.title}\n\n{text}\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    sys.exit(main())
