#!/usr/bin/env python
"""Print the kernel sequence of a rocprofv3 rocpd database around the n-th
dispatch of a named kernel (what runs between two steps).

    python tools/prof_seq.py run_results.db lstm_small_bwd_gs_kernel 30 [window]
"""
import re
import sqlite3
import sys


def main():
    db, pat, nth = sys.argv[1], sys.argv[2], int(sys.argv[3])
    window = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    hits = [i for i, r in enumerate(rows) if re.search(pat, r[0])]
    if len(hits) <= nth + window:
        print("not enough dispatches", len(hits))
        return
    a, b = hits[nth], hits[nth + window]
    t0 = rows[a][1]
    for name, s, e, st in rows[a:b + 1]:
        name = re.sub(r"\(.*", "", name)[:80]
        print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  s{st}  {name}")


if __name__ == "__main__":
    main()
