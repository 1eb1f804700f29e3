#!/usr/bin/env python
"""Aggregate rocprofv3 ``--pmc ... --output-format csv`` counter files per kernel.

    python tools/pmc_summary.py OUT.md DIR [DIR ...]

Every ``*counter_collection.csv`` under the DIRs is read; per (kernel,
counter) the values are summed over dispatches and divided by the dispatch
count (per-dispatch mean), for the kernels matching --match (default: the
framework's own kernels).  Also writes derived ratios where the inputs are
present (VALU busy = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES etc. are left to the
reader: raw per-dispatch means are printed)."""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"(pdrnn::)?\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*", "", name)[:70]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="lstm|slab|adam|gemm|xent|embedding|gru")
    a = ap.parse_args(argv)
    rx = re.compile(a.match)
    rows = []
    for d in a.dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        sums = defaultdict(float)
        disp = defaultdict(set)
        for f in files:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r.get("Kernel_Name", "")
                    if not rx.search(k):
                        continue
                    key = (short(k), r.get("Counter_Name", ""))
                    sums[key] += float(r.get("Counter_Value", 0) or 0)
                    disp[key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        for (k, c), v in sorted(sums.items()):
            n = max(1, len(disp[(k, c)]))
            rows.append((os.path.basename(d.rstrip("/")), k, c, v / n, n))
    with open(a.out, "w") as fh:
        fh.write("| run | kernel | counter | per-dispatch mean | dispatches |\n|---|---|---|---|---|\n")
        for r in rows:
            fh.write(f"| {r[0]} | `{r[1]}` | {r[2]} | {r[3]:.4g} | {r[4]} |\n")
    print(f"{len(rows)} rows -> {a.out}")


if __name__ == "__main__":
    main()
