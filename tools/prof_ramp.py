#!/usr/bin/env python
"""Per-dispatch durations of one kernel over a rocpd trace (warm-up ramp)."""
import re
import sqlite3
import sys

db, pat = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
d = [(s, (e - s) / 1e3) for n, s, e in rows if re.search(pat, n)]
t0 = d[0][0] if d else 0
for i, (s, us) in enumerate(d):
    if i < 12 or i % 10 == 0:
        print(f"{i:4d}  t={(s - t0) / 1e6:9.3f} ms  {us:8.1f} us")
