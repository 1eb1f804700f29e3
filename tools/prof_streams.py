#!/usr/bin/env python
"""Stream/overlap view of a rocprofv3 ``--kernel-trace`` rocpd database.

    python tools/prof_streams.py gpurun_out/x/run_results.db [--match rccl|nccl] [--out profiles/x.md]

Lists, per stream (queue), the kernels and their busy time, then every
matched (communication) kernel with its stream, start/end relative to the
first dispatch, and how many microseconds of OTHER-stream kernels ran while it
was in flight -- the evidence that a bucket all-reduce overlapped compute.
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def _short(name: str, n: int) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"(pdrnn::)?\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:n]


def _cols(c, table):
    return [r[1] for r in c.execute(f"pragma table_info({table})").fetchall()]


def _pick(cols, *names):
    for n in names:
        if n in cols:
            return n
    raise KeyError(f"none of {names} in {cols}")


def analyse(db: str, match: str, limit: int = 40) -> str:
    c = sqlite3.connect(db)
    cols = _cols(c, "kernels")
    st = _pick(cols, "start", "start_ns", "begin")
    en = _pick(cols, "end", "end_ns")
    sid = _pick(cols, "stream_id", "queue_id", "stream")
    rows = c.execute(f"select name, {st}, {en}, {sid} from kernels order by {st}").fetchall()
    if not rows:
        return "no kernels"
    t0 = rows[0][1]
    rx = re.compile(match, re.I)
    per = {}
    for name, s, e, q in rows:
        d = per.setdefault(q, {"n": 0, "busy": 0, "names": {}})
        d["n"] += 1
        d["busy"] += e - s
        k = _short(name, 60)
        d["names"][k] = d["names"].get(k, 0) + 1
    out = [f"database: `{db}`  (stream column `{sid}`)", "", "| stream | dispatches | busy us | top kernels |",
           "|---|---|---|---|"]
    for q, d in sorted(per.items(), key=lambda kv: str(kv[0])):
        top = ", ".join(f"{k} x{n}" for k, n in sorted(d["names"].items(), key=lambda kv: -kv[1])[:4])
        out.append(f"| {q} | {d['n']} | {d['busy'] / 1e3:.1f} | {top} |")
    comm = [r for r in rows if rx.search(r[0])]
    out += ["", f"matched /{match}/: {len(comm)} kernels", "",
            "| # | stream | start us | dur us | other-stream kernel us in flight | concurrent kernels |",
            "|---|---|---|---|---|---|"]
    tot_ov = 0.0
    for i, (name, s, e, q) in enumerate(comm):
        ov, names = 0, {}
        for n2, s2, e2, q2 in rows:
            if q2 == q or s2 >= e or e2 <= s:
                continue
            ov += min(e, e2) - max(s, s2)
            k = _short(n2, 40)
            names[k] = names.get(k, 0) + 1
        tot_ov += ov
        if i < limit:
            out.append(f"| {i} | {q} | {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {ov / 1e3:.1f} | "
                       f"{', '.join(sorted(names))[:80]} |")
    out.append(f"\ntotal other-stream kernel time overlapped by matched kernels: {tot_ov / 1e3:.1f} us")
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="rccl|nccl|allreduce|oneRankReduce")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    txt = analyse(a.db, a.match)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
