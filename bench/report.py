#!/usr/bin/env python
"""Scaling report -- the counterpart of the reference's analysis notebooks
(reference: evaluation/Experiments.ipynb:49-216, Experiments_network.ipynb).

Parses rank 0's ``"0: Memory Usage: M, Training Duration: D"`` line (the same
regex as the notebook) from

* this framework's runner output (JSON Lines, bench/runner.py), and/or
* the reference's published result files (``{"results": [{command, stdout,
  stderr, config}]}``, e.g. /root/reference/evaluation/results_*.json --
  read with the json module only),

and prints markdown tables: epoch time / sequences-per-second / memory per
(trainer, nodes|GPUs, batch), the local baseline, and the speed-up of ours
over the reference for matching configurations.  ``--dedup`` drops the
duplicated ``results_ranks.json`` entries the notebook double-counts
(SURVEY.md §6).  No plotting dependency: ``--csv`` writes the table for any
plotting tool.

    python bench/report.py --ours results/matrix.jsonl \\
        --reference /root/reference/evaluation/results_202007141530.json \\
                    /root/reference/evaluation/results_202007141730.json
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
from collections import defaultdict
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Tuple

PERF = re.compile(r"(\d+): Memory Usage: ([\d.]+), Training Duration: ([\d.]+)")
THRU = re.compile(r"(\d+): Throughput: sequences=(\d+) sequences_per_sec=[\d.]+ world_size=(\d+)")
EPOCH_SEQUENCES = 6912


def _records(path: Path) -> Iterable[Dict]:
    text = Path(path).read_text()
    try:
        obj = json.loads(text)
        if isinstance(obj, dict) and "results" in obj:
            yield from obj["results"]
            return
    except ValueError:
        pass
    for line in text.splitlines():
        line = line.strip()
        if line:
            yield json.loads(line)


def parse_run(rec: Dict) -> Optional[Tuple[str, int, int, float, float, int]]:
    """-> (trainer, nodes/gpus, batch, duration_s, memory_mib, epoch_sequences)
    from rank 0's lines (epoch size from the Throughput line when present,
    else the reference's 6912-sequence training set)."""
    cfg = rec.get("config") or {}
    trainer = cfg.get("trainer") or rec.get("trainer")
    n = cfg.get("gpus") or cfg.get("hosts") or 1
    params = cfg.get("parameters") or {}
    batch = params.get("--batch-size")
    if batch is None:
        m = re.search(r"--batch-size (\d+)", rec.get("command", ""))
        batch = int(m.group(1)) if m else None
    if cfg.get("slots", 1) not in (1, n) and "gpus" not in cfg:
        return None  # reference: only slots == 1 (Experiments.ipynb:77)
    text = (rec.get("stderr") or "") + "\n" + (rec.get("stdout") or "")
    seqs = EPOCH_SEQUENCES
    for m in THRU.finditer(text):
        if m.group(1) == "0":
            seqs = int(m.group(2)) * int(m.group(3))
    for m in PERF.finditer(text):
        if m.group(1) == "0":
            return trainer, int(n), int(batch), float(m.group(3)), float(m.group(2)), seqs
    return None


def aggregate(paths: List[Path], dedup: bool = False) -> Dict[Tuple[str, int, int], Dict[str, float]]:
    seen = set()
    acc: Dict[Tuple[str, int, int], List[Tuple[float, float, int]]] = defaultdict(list)
    for p in paths:
        for rec in _records(p):
            if dedup:
                k = (rec.get("command"), (rec.get("stderr") or "")[-200:])
                if k in seen:
                    continue
                seen.add(k)
            r = parse_run(rec)
            if r:
                acc[r[:3]].append(r[3:])
    out = {}
    for k, v in acc.items():
        d = statistics.mean(x[0] for x in v)
        out[k] = {"duration_s": d, "seq_per_s": statistics.mean(x[2] for x in v) / d,
                  "memory_mib": statistics.mean(x[1] for x in v), "runs": len(v)}
    return out


def table(rows: Dict, title: str) -> str:
    lines = [f"### {title}", "", "| trainer | nodes/GPUs | batch | epoch time (s) | seq/s | memory (MiB) | runs |",
             "|---|---|---|---|---|---|---|"]
    for (tr, n, b), v in sorted(rows.items(), key=lambda kv: (kv[0][0], kv[0][2], kv[0][1])):
        lines.append(f"| {tr} | {n} | {b} | {v['duration_s']:.4f} | {v['seq_per_s']:.1f} | {v['memory_mib']:.1f} | "
                     f"{v['runs']} |")
    return "\n".join(lines)


def compare(ours: Dict, ref: Dict) -> str:
    lines = ["### ours vs reference (matching trainer / count / batch)", "",
             "| trainer | n | batch | ref seq/s | ours seq/s | speed-up |", "|---|---|---|---|---|---|"]
    for k in sorted(set(ours) & set(ref)):
        lines.append(f"| {k[0]} | {k[1]} | {k[2]} | {ref[k]['seq_per_s']:.1f} | {ours[k]['seq_per_s']:.1f} | "
                     f"{ours[k]['seq_per_s'] / ref[k]['seq_per_s']:.0f}x |")
    return "\n".join(lines)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ours", type=Path, nargs="*", default=[])
    ap.add_argument("--reference", type=Path, nargs="*", default=[])
    ap.add_argument("--dedup", action="store_true")
    ap.add_argument("--csv", type=Path, default=None)
    ap.add_argument("--label", default="this framework (MI355X)")
    a = ap.parse_args(argv)
    ours = aggregate(a.ours) if a.ours else {}
    ref = aggregate(a.reference, dedup=a.dedup) if a.reference else {}
    parts = []
    if ref:
        parts.append(table(ref, "reference (Raspberry Pi cluster, published result files)"))
    if ours:
        parts.append(table(ours, a.label))
    if ours and ref:
        parts.append(compare(ours, ref))
    print("\n\n".join(parts))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["source", "trainer", "n", "batch", "duration_s", "seq_per_s", "memory_mib", "runs"])
            for src, rows in (("reference", ref), ("ours", ours)):
                for (tr, n, b), v in sorted(rows.items()):
                    w.writerow([src, tr, n, b, v["duration_s"], v["seq_per_s"], v["memory_mib"], v["runs"]])


if __name__ == "__main__":
    main()
